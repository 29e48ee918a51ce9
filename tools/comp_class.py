#!/usr/bin/env python3
"""Diagnostic: compress / decompress kernel time of a batch of one data class
(3234 x 64 KiB, byU16), round trip checked.  usage: tools/comp_class.py [random|jpeg|text|silesia]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
import lz4e_amd  # noqa: E402
from lz4e_amd import corpus  # noqa: E402

N, BS = 3234, 65536
kind = sys.argv[1] if len(sys.argv) > 1 else "random"
if kind == "random":
    host = np.random.default_rng(7).integers(0, 256, N * BS, dtype=np.uint8)
elif kind == "jpeg":
    host = np.frombuffer((corpus._jpeg() * (N * BS // len(corpus._jpeg()) + 1))[:N * BS], np.uint8).copy()
elif kind == "text":
    host = corpus.text_proxy(N * BS, 7)
else:
    host = corpus.silesia_proxy(N * BS, 0x5157)
dev = torch.device("cuda")
cap = BS + BS // 255 + 16
slot = (cap + 79) // 16 * 16
src = torch.from_numpy(host).to(dev)
offs = torch.arange(N, dtype=torch.int64, device=dev) * BS
lens = torch.full((N,), BS, dtype=torch.int32, device=dev)
tt = torch.full((N,), 1, dtype=torch.uint8, device=dev)
doffs = torch.arange(N, dtype=torch.int64, device=dev) * slot
caps = torch.full((N,), cap, dtype=torch.int32, device=dev)
dst = torch.zeros(N * slot, dtype=torch.uint8, device=dev)
ret = torch.zeros(N, dtype=torch.int32, device=dev)
out = torch.zeros(N * BS + 64, dtype=torch.uint8, device=dev)
dret = torch.zeros(N, dtype=torch.int32, device=dev)
tc, td = [], []
for it in range(8):
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    lz4e_amd.compress_batch_dev(src, offs, lens, tt, dst, doffs, caps, ret, max_len=BS)
    e[1].record()
    lz4e_amd.decompress_batch_dev(dst, doffs, ret, out, offs, lens, dret, max_cap=BS)
    e[2].record()
    torch.cuda.synchronize()
    if it >= 2:
        tc.append(e[0].elapsed_time(e[1]))
        td.append(e[1].elapsed_time(e[2]))
ok = torch.equal(out[:N * BS], src) and bool((dret == BS).all())
r = ret.cpu().numpy().astype(np.int64)
print(f"{kind}: compress {np.mean(tc):.3f} ms, decompress {np.mean(td):.3f} ms, ratio {N * BS / r.sum():.4f}, "
      f"round trip ok={ok}, frames sum {r.sum()}")
