"""Diagnostic: the pipelined 4-wave decoder against the 2-wave streaming
decoder per Silesia-proxy class (kernel times, outputs checked equal to the
input), plus the streaming decoder's per-block cycle counters (stamped
build): parser parse / slot waits, copier record waits, fast and scalar
batches, steps, steps with far (HBM) sources, pointer-jumping rounds.

usage: python tools/streamab.py [blocks per class] [classes,...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import decab  # noqa: E402
from decab import L, corpus  # noqa: E402

SS = ["parse", "p_wait", "c_rec", "c_fast", "c_scalar", "batches", "steps", "far_steps", "rounds",
      "pend_steps"]
PIPE, STREAM = 2, 3


def run(kind, data, bs=65536, cls=1):
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
    decab.lz4e_amd.compress_batch_dev(src, offs, lens, tt, dst, doffs, caps, ret)
    out = torch.zeros(n * bs + 64, dtype=torch.uint8, device=dev)
    dret = torch.zeros(n, dtype=torch.int32, device=dev)
    dbg = torch.zeros(n * decab.NS, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def launch(mode, d=None):
        assert L.lz4e_debug_decompress_stamped(dst.data_ptr(), doffs.data_ptr(), ret.data_ptr(),
                                               out.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                               dret.data_ptr(), n, s, d, bs, mode) == 0

    ms = {}
    for mode in (PIPE, STREAM):
        ts = []
        for _ in range(4):
            out.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch(mode)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
            assert torch.equal(out[:n * bs], src), (kind, mode)
            assert (dret == lens).all().item(), (kind, mode)
        ms[mode] = min(ts[1:])
    launch(STREAM, dbg.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(out[:n * bs], src)
    d = dbg.cpu().numpy().reshape(n, decab.NS).astype(np.float64)
    ratio = n * bs / ret.sum().item()
    print(f"== {kind:8s} {n} x {bs} ratio {ratio:.2f}: pipelined {ms[PIPE]:.3f} ms, streaming "
          f"{ms[STREAM]:.3f} ms ({ms[PIPE] / ms[STREAM]:.2f}x)", flush=True)
    nb = max(1.0, d[:, 5].sum())
    print("   per batch: " + "  ".join(f"{SS[i]} {d[:, i].sum() / nb:.1f}" for i in range(len(SS)) if i != 5)
          + f"  (batches/block {d[:, 5].mean():.0f}, max {d[:, 5].max():.0f})", flush=True)


if __name__ == "__main__":
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    kinds = sys.argv[2].split(",") if len(sys.argv) > 2 else ["text", "ints", "records", "runs", "silesia",
                                                              "text256k"]
    for kind in kinds:
        if kind == "silesia":
            run("silesia", corpus.silesia_proxy(3234 * 65536, 0x5157))
        elif kind == "text256k":
            run("text256k", corpus.text_proxy(953 * 262144, 7), 262144, 3)
        else:
            run(kind, decab.blocks(kind, nb, 65536))
