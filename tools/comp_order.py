"""Diagnostic: compress kernel time of the Silesia-proxy corpus in different
block orders (natural, heaviest classes first, lightest first, interleaved).
Frames are checked identical across orders.  usage: python tools/comp_order.py"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
import lz4e_amd  # noqa: E402
from lz4e_amd import corpus  # noqa: E402

N, BS = 3234, 65536
dev = torch.device("cuda")
sil = corpus.silesia_proxy(N * BS, 0x5157).reshape(N, BS)
cls = np.random.default_rng(0x5157).choice(6, size=N, p=[0.40, 0.15, 0.10, 0.10, 0.10, 0.15])
rank = np.array([2, 0, 3, 5, 4, 1])[cls]  # ints, records, text, runs, jpeg, random
heavy = np.argsort(rank, kind="stable")
inter = np.empty(N, dtype=np.int64)
inter[0::2] = heavy[: (N + 1) // 2]
inter[1::2] = heavy[::-1][: N // 2]
orders = {"natural": np.arange(N), "heavy1st": heavy, "light1st": heavy[::-1], "interleaved": inter}
if os.environ.get("COMP_ORDER_TIERS"):
    # tiers of 1024 blocks (one per SIMD) by measured per-block cycles
    # (tools/stamps.py output), alternately descending and ascending
    cyc = np.load(os.path.join(REPO, "profiles", "r02", "stamps_silesia64k.npy"))
    desc = np.argsort(-cyc, kind="stable")
    T = 1024
    snake = np.concatenate([desc[i:i + T] if (i // T) % 2 == 0 else desc[i:i + T][::-1]
                            for i in range(0, N, T)])
    pair = np.concatenate([desc[:T], desc[::-1][:T], desc[T:N - T]])
    orders = {"measured-desc": desc, "snake": snake, "heavy+lightest": pair}
cap = BS + BS // 255 + 16
slot = (cap + 79) // 16 * 16
offs = torch.arange(N, dtype=torch.int64, device=dev) * BS
lens = torch.full((N,), BS, dtype=torch.int32, device=dev)
tt = torch.full((N,), 1, dtype=torch.uint8, device=dev)
doffs = torch.arange(N, dtype=torch.int64, device=dev) * slot
caps = torch.full((N,), cap, dtype=torch.int32, device=dev)
ref = None
for name, o in orders.items():
    src = torch.from_numpy(np.ascontiguousarray(sil[o]).reshape(-1)).to(dev)
    dst = torch.zeros(N * slot, dtype=torch.uint8, device=dev)
    ret = torch.zeros(N, dtype=torch.int32, device=dev)
    ts = []
    for _ in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lz4e_amd.compress_batch_dev(src, offs, lens, tt, dst, doffs, caps, ret)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    r = ret.cpu().numpy()
    inv = np.empty(N, dtype=np.int64)
    inv[o] = np.arange(N)
    sizes = r[inv]
    if ref is None:
        ref = sizes
    assert (sizes == ref).all(), name
    print(f"{name:12s} compress {min(ts[1:]):.3f} ms (median {np.median(ts[1:]):.3f})", flush=True)
