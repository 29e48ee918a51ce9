#!/usr/bin/env python3
"""Step pipelining experiment: the bench's serial step (compress then
decompress on one stream) against a two-stream pipeline in which batch s's
decompress overlaps batch s+1's compress (double-buffered frame slots).
Prints ms per step for each schedule; every schedule's last round trip is
checked.  tools/pipe_exp.py [--workload silesia64k] [--steps 20]"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import lz4e_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="silesia64k")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    bs, cls, gen, _, _ = bench.WORKLOADS[a.workload]
    nblk = bench.DEFAULT_BLOCKS[a.workload]
    dev = torch.device("cuda:0")
    host = bench.make_data(gen, nblk * bs, bench.CORPUS_SEED)
    lens = [bs] * nblk
    d_src = torch.from_numpy(host).to(dev)
    b = bench.Batch(d_src, lens, bs, cls, dev)
    dst2 = [b.d_dst, torch.zeros_like(b.d_dst)]
    ret2 = [b.d_ret, torch.zeros_like(b.d_ret)]

    def comp(i, st):
        lz4e_amd.compress_batch_dev(b.d_src, b.d_off, b.d_len, b.d_tt, dst2[i], b.d_doff, b.d_cap,
                                    ret2[i], max_len=bs, stream=st.cuda_stream)

    def dec(i, st):
        lz4e_amd.decompress_batch_dev(dst2[i], b.d_doff, ret2[i], b.d_out, b.d_off, b.d_len, b.d_dret,
                                      stream=st.cuda_stream, max_cap=b.max_cap)

    def serial(K):
        st = torch.cuda.current_stream(dev)
        for _ in range(K):
            comp(0, st)
            dec(0, st)

    def piped(K, pa, pb):
        A = torch.cuda.Stream(dev, priority=pa)
        B = torch.cuda.Stream(dev, priority=pb)
        cur = torch.cuda.current_stream(dev)
        A.wait_stream(cur)
        B.wait_stream(cur)
        cdone = [torch.cuda.Event() for _ in range(K)]
        ddone = [torch.cuda.Event() for _ in range(K)]
        for s in range(K):
            if s >= 2:
                A.wait_event(ddone[s - 2])
            comp(s % 2, A)
            cdone[s].record(A)
            B.wait_event(cdone[s])
            dec(s % 2, B)
            ddone[s].record(B)
        cur.wait_stream(A)
        cur.wait_stream(B)

    def timeit(f, K):
        f(2)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        f(K)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) * 1e3 / K

    lo, hi = torch.cuda.Stream.priority_range()
    print(f"stream priority range {lo}..{hi}")
    U = b.U
    for name, f in [("serial", serial),
                    ("piped A=hi B=lo", lambda K: piped(K, hi, lo)),
                    ("piped equal", lambda K: piped(K, 0, 0)),
                    ("piped A=lo B=hi", lambda K: piped(K, lo, hi)),
                    ("serial again", serial)]:
        ms = timeit(f, a.steps)
        ok = torch.equal(b.d_out[:U], b.d_src[:U]) and bool((b.d_dret.cpu().numpy() == bs).all())
        print(f"{a.workload} {name:18s} {ms:7.3f} ms/step  {U / ms / 1e-3 / 2**30:7.2f} GiB/s  ok={ok}",
              flush=True)


if __name__ == "__main__":
    main()
