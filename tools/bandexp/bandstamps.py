"""Diagnostic: the band compressor's per-phase cycles (stamped build).

python tools/bandstamps.py [silesia|text256k|fio4k] [nblocks]

Runs lz4e_debug_compress_band over the workload (all blocks, and the 4 blocks
with the most passes alone), prints thread 0's shader cycles per phase per
block (fill, cands, verify, commit, hits, chain), the chain passes and
commits per block, and the kernel times of the unstamped band and wave
compressors (HIP events, LZ4E_COMPRESS_MODE is read once per process, so the
wave time comes from lz4e_debug_compress_stamped's unstamped sibling: the
stamped one-wave kernel is not timed here).
"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
import lz4e_amd  # noqa: E402
from lz4e_amd import corpus  # noqa: E402

lz4e_amd.lib()  # (HIP runtime up)
L = ctypes.CDLL(os.environ.get("BAND_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libband.so")))
P = ctypes.c_void_p
L.band_compress_dev.argtypes = [P] * 8 + [ctypes.c_uint32, ctypes.c_uint32, P, P]
L.band_compress_dev.restype = ctypes.c_int
PH = ["fill", "cands", "verify", "commit", "hits", "chain"]


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "silesia"
    nmax = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 30
    if wl == "text256k":
        bs, cls, data = 262144, 3, corpus.text_proxy(3815 * 262144, 0x7E57)
    elif wl == "fio4k":
        bs, cls, data = 4096 * 2, 1, corpus.fio_pattern(65536 * 4096)
    else:
        bs, cls, data = 65536, 1, corpus.silesia_proxy(3234 * 65536, 0x5157)
    n = min(data.size // bs, nmax)
    dev = torch.device("cuda")
    offs = torch.arange(n, dtype=torch.int64, device=dev) * bs
    lens = torch.full((n,), bs, dtype=torch.int32, device=dev)
    tt = torch.full((n,), cls, dtype=torch.uint8, device=dev)
    cap = bs + bs // 255 + 16
    slot = (cap + 79) // 16 * 16
    doffs = torch.arange(n, dtype=torch.int64, device=dev) * slot
    caps = torch.full((n,), cap, dtype=torch.int32, device=dev)
    src = torch.from_numpy(np.ascontiguousarray(data[:n * bs])).to(dev)
    dst = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    ret = torch.zeros(n, dtype=torch.int32, device=dev)
    dbg = torch.zeros(n * 16, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def stamped(sl=slice(None), k=n):
        dbg.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = L.band_compress_dev(src.data_ptr(), offs[sl].data_ptr(), lens[sl].data_ptr(), tt[sl].data_ptr(),
                                       dst.data_ptr(), doffs[sl].data_ptr(), caps[sl].data_ptr(), ret[sl].data_ptr(),
                                       k, bs, s, dbg.data_ptr())
        e1.record()
        assert r == 0
        torch.cuda.synchronize()
        return e0.elapsed_time(e1), dbg[:16 * k].cpu().numpy().reshape(k, 16).astype(np.float64)

    stamped()
    ms, d = stamped()
    print(f"{wl}: {n} blocks x {bs} B, stamped band kernel (+prev_kernel) {ms:.3f} ms")
    tot = d[:, :6].sum(1)
    print(f"  cycles per block: mean {tot.mean():.0f} max {tot.max():.0f}; chain passes mean {d[:, 6].mean():.1f} "
          f"max {d[:, 6].max():.0f}; commits mean {d[:, 7].mean():.1f}")
    per = d[:, :6].sum(0) / max(d[:, 6].sum(), 1)
    print("  cycles per chain pass: " + ", ".join(f"{PH[i]} {per[i]:.0f}" for i in range(6)) +
          f"  (total {per.sum():.0f})")
    CH = ["masks", "entry", "next", "doubling", "stitch", "end", "nodescan", "flags"]
    chs = d[:, 8:16].sum(0) / max(d[:, 6].sum(), 1)
    print("  chain split per pass: " + ", ".join(f"{CH[i]} {chs[i]:.0f}" for i in range(8)))
    if wl == "silesia":
        names = ["text", "ints", "runs", "random", "jpeg", "records"]
        cls_of = np.random.default_rng(0x5157).choice(6, size=3234, p=[0.40, 0.15, 0.10, 0.10, 0.10, 0.15])[:n]
        for c in range(6):
            m = cls_of == c
            if m.any():
                pc = d[m, :6].sum(0) / max(d[m, 6].sum(), 1)
                print(f"  {names[c]:8s} n={m.sum():4d} cycles/block {tot[m].mean():10.0f} max {tot[m].max():10.0f} "
                      f"passes {d[m, 6].mean():6.1f}; per pass " + ", ".join(f"{PH[i]} {pc[i]:.0f}" for i in range(6)))
        texts = np.nonzero(cls_of == 0)[0]
        if texts.size:
            i = int(texts[0])
            msi, di = stamped(slice(i, i + 1), 1)
            pp = di[0, :6] / max(di[0, 6], 1)
            print(f"  text block {i} alone: {msi:.3f} ms, {di[0, :6].sum():.0f} cycles, passes {di[0, 6]:.0f}; per pass "
                  + ", ".join(f"{PH[k]} {pp[k]:.0f}" for k in range(6)))
            cs = di[0, 8:16] / max(di[0, 6], 1)
            print("    chain split: " + ", ".join(f"{CH[k]} {cs[k]:.0f}" for k in range(8)))
    order = np.argsort(d[:, 6])[::-1][:4]
    for i in order:
        i = int(i)
        msi, di = stamped(slice(i, i + 1), 1)
        t = di[0, :6].sum()
        pp = di[0, :6] / max(di[0, 6], 1)
        print(f"  block {i} alone: {msi:.3f} ms, {t:.0f} cycles, passes {di[0, 6]:.0f} (full launch "
              f"{d[i, :6].sum():.0f} cycles); per pass " + ", ".join(f"{PH[k]} {pp[k]:.0f}" for k in range(6)))


if __name__ == "__main__":
    main()
