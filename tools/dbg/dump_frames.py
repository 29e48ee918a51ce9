"""Debug: re-run one parametrized batch case of test_compress_batch_vs_oracle
on the GPU and save every block + GPU frame under gpurun_out/dbg/ (offline
diff against the oracle with tools/dbg/diff_frames.py)."""
import os
import sys
import zlib

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "lz4-sgori_amd")]
import lz4e_amd  # noqa
import test_gpu_parity as T  # noqa

kind, cls = sys.argv[1], int(sys.argv[2])
rng = np.random.default_rng(zlib.crc32(f"{kind}-{cls}".encode()))
data = T._corpus(kind, 1 << 21, 17)
lens = [int(x) for x in rng.choice([0, 1, 12, 13, 14, 100, 4096, 4097, 30000, 65535, 65536], size=48)]
if cls == 3:
    lens += [65537, 131072, 200000]
blocks = []
for ln in lens:
    s = int(rng.integers(0, data.size - ln))
    blocks.append(data[s:s + ln].tobytes())
r, frames, aux = T._gpu_compress(lz4e_amd, blocks, [cls] * len(blocks))
out = os.path.join(REPO, "gpurun_out", "dbg")
os.makedirs(out, exist_ok=True)
for i, b in enumerate(blocks):
    open(os.path.join(out, f"{kind}_{cls}_{i}.in"), "wb").write(b)
    open(os.path.join(out, f"{kind}_{cls}_{i}.gpu"), "wb").write(bytes(frames[i]))
print("saved", len(blocks))
