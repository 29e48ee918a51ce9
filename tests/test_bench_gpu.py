"""bench.py's measurement legs on a small batch (GPU): the decompress-only
leg of configs[4] and the per-block floor, through the same functions the
bench line uses, on 256 KiB text blocks -- sizes decoded exact, the bytes
equal to the input, the lines well formed."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def text_batch():
    import torch
    import bench
    import lz4e_amd
    if not lz4e_amd.gpu_available():
        pytest.fail("HIP path unavailable: " + lz4e_amd.last_error())
    dev = torch.device("cuda:0")
    bs, nblk = 262144, 48
    lens = np.full(nblk, bs, dtype=np.int64)
    lens[-1] = 182784  # the enwik9 layout's short last block
    host = np.zeros(nblk * bs, np.uint8)
    host[:int(lens.sum())] = bench.make_data("text", int(lens.sum()), 11)
    b = bench.Batch(torch.from_numpy(host).to(dev), lens, bs, lz4e_amd.BYU32, dev)
    b.run(1, False)
    b.check_roundtrip()
    return b, dev


def test_decompress_only_leg(text_batch):
    import torch
    import bench
    b, dev = text_batch
    b.d_out.zero_()
    b.d_dret.zero_()
    out = bench.decompress_only(b, 3, 0, 1, None, dev, "", "text256k")
    assert (b.d_dret.cpu().numpy() == b.lens).all()
    n = int(b.lens.sum())
    assert torch.equal(b.d_out[:n], b.d_src[:n])
    w, s = out["weak"], out["strong"]
    assert out["kernel"] == "decompress" and w["value"] > 0 and w["ms_per_step"] > 0
    assert w["roofline"]["algorithmic_bytes_per_launch"] == n + int(b.rets.astype(np.int64).sum())
    assert 0 < w["roofline"]["frac"] < 1
    # one rank: the strong job is the whole batch
    assert s["blocks_this_rank"] == b.nblk and s["value"] > 0


def test_block_floor_leg(text_batch):
    import bench
    b, _ = text_batch
    f = bench.block_floor(b, top=2, reps=2)
    assert f["floor_ms"] > 0 and f["compress_ms"] > 0 and f["decompress_ms"] > 0
    assert (b.d_dret.cpu().numpy() == b.lens).all()
