"""Diagnostic: the wide decoder's stamped build (lz4e_debug_decompress_stamped,
mode 8): per block the chunks, assembly steps, pointer rounds, exact
sequences and walker re-walks, and thread 0's cycles per phase (stage,
token starts, fields + checks, byte classification, pointer rounds, stores,
exact sequences); printed as means over the blocks and for the slowest block.

usage: python tools/widestamps.py [workloads, e.g. text,silesia,text256k]"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import lz4e_amd  # noqa: E402
from decmodes import class_blocks  # noqa: E402
from lz4e_amd import corpus  # noqa: E402

L = lz4e_amd.lib()
P = ctypes.c_void_p
L.lz4e_debug_decompress_stamped.argtypes = [P] * 7 + [ctypes.c_uint32, P, P, ctypes.c_uint32,
                                                       ctypes.c_uint32]
PH = ["stage", "starts", "fields", "classify", "rounds", "store", "exact"]


def run(name, data, bs, cls):
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
    dbg = torch.zeros(n * 16, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        dbg.zero_()
        assert L.lz4e_debug_decompress_stamped(dst.data_ptr(), doffs.data_ptr(), ret.data_ptr(), out.data_ptr(),
                                               offs.data_ptr(), lens.data_ptr(), dret.data_ptr(), n, s,
                                               dbg.data_ptr(), bs, 8) == 0
        torch.cuda.synchronize()
    ok = torch.equal(out[:n * bs], src) and bool((dret == lens).all().item())
    d = dbg.view(n, 16).cpu().numpy().astype(np.float64)
    tot = d[:, 8:15].sum(1)
    w = int(np.argmax(tot))
    print(f"== {name} {n} x {bs} {'ok' if ok else 'MISMATCH'}: per block chunks {d[:, 0].mean():.1f} steps "
          f"{d[:, 1].mean():.1f} rounds {d[:, 2].mean():.1f} exact {d[:, 3].mean():.2f} rewalks {d[:, 4].mean():.2f}; "
          f"cycles mean {tot.mean() / 1e3:.0f} k, max {tot[w] / 1e3:.0f} k", flush=True)
    print("   mean per block: " + ", ".join(f"{p} {d[:, 8 + i].mean() / 1e3:.1f} k" for i, p in enumerate(PH)))
    c = max(d[:, 0].mean(), 1)
    print("   mean per chunk: " + ", ".join(f"{p} {d[:, 8 + i].mean() / c:.0f}" for i, p in enumerate(PH)))
    print(f"   slowest block {w}: chunks {d[w, 0]:.0f} steps {d[w, 1]:.0f} rounds {d[w, 2]:.0f} exact {d[w, 3]:.0f} "
          f"rewalks {d[w, 4]:.0f}; " + ", ".join(f"{p} {d[w, 8 + i] / 1e3:.1f} k" for i, p in enumerate(PH)),
          flush=True)


if __name__ == "__main__":
    wls = (sys.argv[1] if len(sys.argv) > 1 else "text,random,silesia").split(",")
    for kind in ("text", "ints", "records", "runs", "random", "jpeg"):
        if kind in wls:
            run(kind, class_blocks(kind, 256, 65536), 65536, 1)
    if "silesia" in wls:
        run("silesia64k", corpus.silesia_proxy(3234 * 65536, 0x5157), 65536, 1)
    if "text256k" in wls:
        run("text256k", corpus.text_proxy(3815 * 262144, 0x7E57), 262144, 3)
