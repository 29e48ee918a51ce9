"""Workload for SQ counter passes per Silesia-proxy class: compress (then
decompress) 256 blocks of 64 KiB of one class, once.
usage: python tools/sq_class.py <text|ints|records>"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import lz4e_amd  # noqa: E402
from decab import blocks  # noqa: E402

kind = sys.argv[1]
n, bs = 256, 65536
data = blocks(kind, n, bs)
dev = torch.device("cuda")
offs = torch.arange(n, dtype=torch.int64, device=dev) * bs
lens = torch.full((n,), bs, dtype=torch.int32, device=dev)
tt = torch.full((n,), 1, dtype=torch.uint8, device=dev)
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
lz4e_amd.decompress_batch_dev(dst, doffs, ret, out, offs, lens, dret)
torch.cuda.synchronize()
assert torch.equal(out[:n * bs], src)
print(kind, "ok", int(ret.sum()))
