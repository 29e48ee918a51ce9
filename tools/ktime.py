"""Diagnostic: kernel time of compress (and decompress) on fixed workloads,
for A/B-ing builds (LZ4E_LIB=...).  Prints one line per workload."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
import lz4e_amd  # noqa
from lz4e_amd import corpus  # noqa


def run(name, data, bs, reps=5, cls=None):
    dev = torch.device("cuda")
    n = data.size // bs
    offs = torch.arange(n, dtype=torch.int64, device=dev) * bs
    lens = torch.full((n,), bs, dtype=torch.int32, device=dev)
    tt = torch.full((n,), cls or (1 if bs <= 65536 else 3), dtype=torch.uint8, device=dev)
    cap = bs + bs // 255 + 16
    slot = (cap + 79) // 16 * 16
    doffs = torch.arange(n, dtype=torch.int64, device=dev) * slot
    caps = torch.full((n,), cap, dtype=torch.int32, device=dev)
    src = torch.from_numpy(data).to(dev)
    dst = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    ret = torch.zeros(n, dtype=torch.int32, device=dev)
    out = torch.zeros(n * bs + 64, dtype=torch.uint8, device=dev)
    dret = torch.zeros(n, dtype=torch.int32, device=dev)
    tc, td = [], []
    for i in range(reps + 1):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        lz4e_amd.compress_batch_dev(src, offs, lens, tt, dst, doffs, caps, ret)
        e1.record()
        lz4e_amd.decompress_batch_dev(dst, doffs, ret, out, offs, lens, dret)
        e2.record()
        torch.cuda.synchronize()
        if i:
            tc.append(e0.elapsed_time(e1))
            td.append(e1.elapsed_time(e2))
    ok = bool((dret == lens).all()) and torch.equal(out[: n * bs], src)
    print(f"{name:12s} compress {np.median(tc):8.3f} ms  decompress {np.median(td):7.3f} ms  "
          f"ratio {n * bs / ret.sum().item():.4f} roundtrip_ok={ok}", flush=True)


if __name__ == "__main__":
    tag = os.environ.get("LZ4E_LIB", "default")
    print("==", tag)
    run("silesia64k", corpus.silesia_proxy(3234 * 65536, 0x5157), 65536)
    if os.environ.get("KTIME_T256"):  # configs[4]: 3 815 blocks of 256 KiB (byU32), issue-bound
        run("text256k", corpus.text_proxy(3815 * 262144, 7), 262144)
    if os.environ.get("KTIME_U32"):  # the sg512 workload's table class
        run("silesia64k-u32", corpus.silesia_proxy(3234 * 65536, 0x5157), 65536, cls=3)
    run("text64k", corpus.text_proxy(1024 * 65536, 7), 65536)
    run("fio4k", corpus.fio_pattern(262144 * 4096), 4096)
    run("text4k", corpus.text_proxy(16384 * 4096, 9), 4096)
