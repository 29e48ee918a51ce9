"""Diagnostic: decoder kernels side by side -- the one-wave decoder (1), the
pipelined 4-wave decoder (2) and the chunked decoder (4) on the same frames
(compressed on the GPU), kernel time by HIP events (median of the timed
launches after one warm-up; outputs checked equal to the input and the
return values to the block sizes).

usage: python tools/decmodes.py [modes, e.g. 2,4] [workloads, e.g. silesia,text256k,fio4k,classes]"""
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
NAMES = {1: "one-wave", 2: "pipelined", 6: "lds-small", 7: "group"}


def class_blocks(kind, n, bs):
    rng = np.random.default_rng(5)
    jpg = np.frombuffer(corpus._jpeg(), np.uint8)
    gen = {"text": lambda: corpus.text_proxy(bs, int(rng.integers(1 << 30))),
           "ints": lambda: corpus._int_table(bs, rng), "records": lambda: corpus._records(bs, rng),
           "runs": lambda: corpus._runs(bs, rng),
           "random": lambda: rng.integers(0, 256, bs, dtype=np.uint8),
           "jpeg": lambda: jpg[(s := int(rng.integers(0, jpg.size - bs))):s + bs]}[kind]
    return np.concatenate([gen() for _ in range(n)])


def run(name, data, bs, cls, modes, reps=5):
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
    torch.cuda.synchronize()
    out = torch.zeros(n * bs + 64, dtype=torch.uint8, device=dev)
    dret = torch.zeros(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    csum = ret.sum().item()
    res = {}
    for mode in modes:
        ts = []
        for r in range(reps + 1):
            out.zero_()
            dret.fill_(-12345)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert L.lz4e_debug_decompress_stamped(dst.data_ptr(), doffs.data_ptr(), ret.data_ptr(),
                                                   out.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                                   dret.data_ptr(), n, s, None, bs, mode) == 0
            e1.record()
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
            ok = torch.equal(out[:n * bs], src) and bool((dret == lens).all().item())
            if not ok:
                bad = (dret != lens).nonzero().flatten()[:5].tolist()
                print(f"!! {name} mode {mode}: MISMATCH (ret bad blocks {bad})", flush=True)
                return
        res[mode] = float(np.median(ts))
    gbs = {m: (n * bs + csum) / (t * 1e-3) / 1e9 for m, t in res.items()}
    print(f"== {name:10s} {n} x {bs} ratio {n * bs / csum:.2f}: " +
          ", ".join(f"{NAMES[m]} {t:.3f} ms ({gbs[m]:.0f} GB/s U+C, {gbs[m] / 8000:.3f} of HBM)"
                    for m, t in res.items()), flush=True)


if __name__ == "__main__":
    modes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,4").split(",")]
    wls = (sys.argv[2] if len(sys.argv) > 2 else "silesia,text256k,fio4k,classes").split(",")
    if "classes" in wls:
        for kind in ("text", "ints", "records", "runs", "random", "jpeg"):
            run(kind, class_blocks(kind, 256, 65536), 65536, 1, modes)
    if "silesia" in wls:
        run("silesia64k", corpus.silesia_proxy(3234 * 65536, 0x5157), 65536, 1, modes)
    if "text256k" in wls:
        run("text256k", corpus.text_proxy(3815 * 262144, 0x7E57), 262144, 3, modes)
    if "fio4k" in wls:
        run("fio4k", corpus.fio_pattern(262144 * 4096), 4096, 1, modes)
    if "sil4k_1k" in wls:  # a batch of 1 024 small blocks (decoder choice for mid-size batches)
        run("sil4k_1k", corpus.silesia_proxy(1024 * 4096, 0x5157), 4096, 1, modes)
    if "fio4k_1k" in wls:
        run("fio4k_1k", corpus.fio_pattern(1024 * 4096), 4096, 1, modes)
    if "sil4k_3k" in wls:
        run("sil4k_3k", corpus.silesia_proxy(3072 * 4096, 0x5157), 4096, 1, modes)
    for nb in (4096, 16384, 65536):  # fio blocks in mid-size batches (lane / group thresholds)
        if f"fio4k_{nb // 1024}k" in wls:
            run(f"fio4k_{nb // 1024}k", corpus.fio_pattern(nb * 4096), 4096, 1, modes)
    if "sil4k" in wls:  # short sequences in small blocks
        run("sil4k", corpus.silesia_proxy(65536 * 4096, 0x5157), 4096, 1, modes)
