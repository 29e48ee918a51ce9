"""Diagnostic: compress (and decompress) of one Silesia-proxy class only, for
rocprofv3 --pmc instruction-mix runs.  usage: python tools/sq_class.py CLASS [blocks]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
import lz4e_amd  # noqa
from lz4e_amd import corpus  # noqa

kind = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
bs = 65536
rng = np.random.default_rng(5)
gen = {"text": lambda m: corpus.text_proxy(m, 3), "ints": lambda m: corpus._int_table(m, rng),
       "records": lambda m: corpus._records(m, rng), "runs": lambda m: corpus._runs(m, rng)}[kind]
data = np.concatenate([gen(bs) for _ in range(n)])
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
out = torch.zeros(n * bs + 64, dtype=torch.uint8, device=dev)
dret = torch.zeros(n, dtype=torch.int32, device=dev)
for _ in range(2):
    lz4e_amd.compress_batch_dev(src, offs, lens, tt, dst, doffs, caps, ret)
    lz4e_amd.decompress_batch_dev(dst, doffs, ret, out, offs, lens, dret)
torch.cuda.synchronize()
assert torch.equal(out[:n * bs], src)
print(kind, n, "ratio", n * bs / ret.sum().item())
