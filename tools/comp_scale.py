"""Diagnostic: compress kernel time of N text blocks (64 KiB) for N = 256 ..
2560 (1 .. 10 per CU): how a block's parse slows with co-resident blocks.
usage: python tools/comp_scale.py"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
import lz4e_amd  # noqa: E402
from lz4e_amd import corpus  # noqa: E402

BS = 65536
dev = torch.device("cuda")
text = corpus.text_proxy(2560 * BS, 7)
for N in (256, 512, 1024, 1536, 2048, 2560):
    offs = torch.arange(N, dtype=torch.int64, device=dev) * BS
    lens = torch.full((N,), BS, dtype=torch.int32, device=dev)
    tt = torch.full((N,), 1, dtype=torch.uint8, device=dev)
    cap = BS + BS // 255 + 16
    slot = (cap + 79) // 16 * 16
    doffs = torch.arange(N, dtype=torch.int64, device=dev) * slot
    caps = torch.full((N,), cap, dtype=torch.int32, device=dev)
    src = torch.from_numpy(text[:N * BS]).to(dev)
    dst = torch.zeros(N * slot, dtype=torch.uint8, device=dev)
    ret = torch.zeros(N, dtype=torch.int32, device=dev)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lz4e_amd.compress_batch_dev(src, offs, lens, tt, dst, doffs, caps, ret)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(f"text x {N:5d} ({N / 256:.1f} per CU): compress {min(ts[1:]):.3f} ms", flush=True)
