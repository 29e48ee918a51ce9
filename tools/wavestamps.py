"""Diagnostic: the one-wave decoder's stamped cycle counters per block
(parse, fast-batch loads + span setup, copies / dependency rounds, store
pass; batches and rounds), means over the blocks of a workload, for the
modes given (1: one-wave, 6: its LDS form for small blocks).

usage: python tools/wavestamps.py [modes, e.g. 1,6] [workloads, e.g. fio4k,silesia]"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
import lz4e_amd  # noqa: E402
from lz4e_amd import corpus  # noqa: E402

L = lz4e_amd.lib()
P = ctypes.c_void_p
L.lz4e_debug_decompress_stamped.argtypes = [P] * 7 + [ctypes.c_uint32, P, P, ctypes.c_uint32,
                                                       ctypes.c_uint32]


def run(name, data, bs, cls, modes):
    dev = torch.device("cuda")
    n = data.size // bs
    offs = torch.arange(n, dtype=torch.int64, device=dev) * bs
    lens = torch.full((n,), bs, dtype=torch.int32, device=dev)
    tt = torch.full((n,), cls, dtype=torch.uint8, device=dev)
    cap = bs + bs // 255 + 16
    slot = (cap + 79) // 16 * 16
    doffs = torch.arange(n, dtype=torch.int64, device=dev) * slot
    caps = torch.full((n,), cap, dtype=torch.int32, device=dev)
    src = torch.from_numpy(data).to(dev)
    dst = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    ret = torch.zeros(n, dtype=torch.int32, device=dev)
    lz4e_amd.compress_batch_dev(src, offs, lens, tt, dst, doffs, caps, ret)
    out = torch.zeros(n * bs + 64, dtype=torch.uint8, device=dev)
    dret = torch.zeros(n, dtype=torch.int32, device=dev)
    dbg = torch.zeros(n * 8, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for mode in modes:
        for _ in range(2):
            dbg.zero_()
            assert L.lz4e_debug_decompress_stamped(dst.data_ptr(), doffs.data_ptr(), ret.data_ptr(),
                                                   out.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                                   dret.data_ptr(), n, s, dbg.data_ptr(), bs, mode) == 0
            torch.cuda.synchronize()
        assert torch.equal(out[:n * bs], src) and bool((dret == lens).all().item())
        d = dbg.view(n, 8).cpu().numpy().astype(np.float64)
        if mode == 7:  # group decoder: no per-block stamps (only the resumed blocks' one-wave stamps)
            print(f"== {name} mode 7 (group decoder): handed-over blocks' one-wave stamps only", flush=True)
        tot = d[:, 0] + d[:, 1] + d[:, 2] + d[:, 5]
        print(f"== {name} mode {mode}: cycles/block mean {tot.mean():.0f} (p90 {np.percentile(tot, 90):.0f}): "
              f"parse {d[:, 0].mean():.0f}, loads+span {d[:, 1].mean():.0f}, copies/rounds {d[:, 2].mean():.0f}, "
              f"store {d[:, 5].mean():.0f}; batches {d[:, 3].mean():.1f}, rounds {d[:, 4].mean():.1f}",
              flush=True)


if __name__ == "__main__":
    modes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,6").split(",")]
    wls = (sys.argv[2] if len(sys.argv) > 2 else "fio4k").split(",")
    if "fio4k" in wls:
        run("fio4k", corpus.fio_pattern(262144 * 4096), 4096, 1, modes)
    if "sil4k" in wls:
        run("sil4k", corpus.silesia_proxy(65536 * 4096, 0x5157), 4096, 1, modes)
    if "silesia" in wls:
        run("silesia64k", corpus.silesia_proxy(3234 * 65536, 0x5157), 65536, 1, modes)
