"""Diagnostic: round trip of the silesia64k batch split over S streams (each
part: compress launch then decompress launch on its own stream; streams
alternate priority so they land on distinct hardware queues)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
import lz4e_amd  # noqa
from lz4e_amd import corpus  # noqa


def main():
    dev = torch.device("cuda")
    bs, n = 65536, 3234
    data = corpus.silesia_proxy(n * bs, 0x5157)
    src = torch.from_numpy(data).to(dev)
    cap = bs + bs // 255 + 16
    slot = (cap + 79) // 16 * 16
    dst = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    out = torch.zeros(n * bs + 64, dtype=torch.uint8, device=dev)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    for S in (1, 2, 4, 8):
        for mode in ("contig", "interleave"):
            idx = [np.arange(n)[p::S] if mode == "interleave" else np.array_split(np.arange(n), S)[p]
                   for p in range(S)]
            parts = []
            for p in range(S):
                i = torch.from_numpy(idx[p]).to(dev)
                m = i.numel()
                parts.append(dict(
                    offs=(i * bs).to(torch.int64), lens=torch.full((m,), bs, dtype=torch.int32, device=dev),
                    tt=torch.ones(m, dtype=torch.uint8, device=dev), doffs=(i * slot).to(torch.int64),
                    caps=torch.full((m,), cap, dtype=torch.int32, device=dev),
                    ret=torch.zeros(m, dtype=torch.int32, device=dev), dret=torch.zeros(m, dtype=torch.int32, device=dev),
                    st=torch.cuda.Stream(priority=-1 if p % 2 else 0)))
            times = []
            for rep in range(4):
                out.zero_()
                torch.cuda.synchronize()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for q in parts:
                    q["st"].wait_event(e0)
                for q in parts:
                    lz4e_amd.compress_batch_dev(src, q["offs"], q["lens"], q["tt"], dst, q["doffs"], q["caps"],
                                                q["ret"], max_len=bs, stream=q["st"].cuda_stream)
                    lz4e_amd.decompress_batch_dev(dst, q["doffs"], q["ret"], out, q["offs"], q["lens"], q["dret"],
                                                  stream=q["st"].cuda_stream)
                for q in parts:
                    torch.cuda.current_stream().wait_stream(q["st"])
                e1.record()
                torch.cuda.synchronize()
                if rep:
                    times.append(e0.elapsed_time(e1))
            ok = torch.equal(out[:n * bs], src) and all(bool((q["dret"] == bs).all()) for q in parts)
            t = float(np.median(times))
            print(f"S={S} {mode:10s} step {t:7.3f} ms  {n * bs / t / 1e3 / 2**30 * 1e6:7.2f} GiB/s ok={ok}", flush=True)


main()
