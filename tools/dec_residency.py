"""Decoder residency probe (silesia64k): decompress time of the k heaviest
blocks alone (heaviest = most compressed bytes, the decoder's own launch
weight) for growing k.  If the kernel time grows in steps at multiples of
the resident workgroup count (6 per CU = 1 536), the launch is bound by
rounds of blocks, not by one block's chain.

  python tools/dec_residency.py [--reps 10]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))


def main():
    import torch
    import bench
    import lz4e_amd
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    bs, nblk = 65536, 3234
    host = bench.make_data("silesia", bs * nblk, 0)
    d_src = torch.from_numpy(host).to(dev)
    b = bench.Batch(d_src, [bs] * nblk, bs, lz4e_amd.BYU16, dev)
    b.compress()
    torch.cuda.synchronize()
    rets = b.d_ret.cpu().numpy()
    order = np.argsort(-rets, kind="stable")
    st = b.stream
    res = {}
    for k in (128, 256, 512, 768, 1024, 1280, 1536, 1792, 2048, 2304, 2560, 3234):
        idx = torch.from_numpy(order[:k].astype(np.int64)).to(dev)
        doff, dret_in = b.d_doff[idx].contiguous(), b.d_ret[idx].contiguous()
        off, ln = b.d_off[idx].contiguous(), b.d_len[idx].contiguous()
        dret = torch.zeros(k, dtype=torch.int32, device=dev)
        ts = []
        for r in range(args.reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            lz4e_amd.decompress_batch_dev(b.d_dst, doff, dret_in, b.d_out, off, ln, dret,
                                          stream=st.cuda_stream, max_cap=bs)
            e1.record(st)
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(e0.elapsed_time(e1))
        assert (dret.cpu().numpy() == bs).all()
        res[k] = round(float(np.median(ts)), 4)
        print(f"k={k:5d} decompress {res[k]:.4f} ms  (mean frame {rets[order[:k]].mean():.0f} B)",
              flush=True)
    print(json.dumps({"decode_ms_by_heaviest_k": res}))


if __name__ == "__main__":
    main()
