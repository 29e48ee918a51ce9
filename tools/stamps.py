"""Diagnostic: per-phase cycle breakdown of the compress kernel (stamped build).

Runs lz4e_debug_compress_stamped over a workload and prints, per block class,
the mean cycles per block spent in each phase plus sequence counts.
"""
import ctypes
import os
import sys

import numpy as np

CLASS_NAMES = ["text", "ints", "runs", "random", "jpeg", "records"]

def by_class(name, tot, n, extra=None):
    if not name.startswith("silesia"):
        return
    cls = np.random.default_rng(0x5157).choice(6, size=n, p=[0.40, 0.15, 0.10, 0.10, 0.10, 0.15])
    for c in range(6):
        m = cls == c
        if m.any():
            print(f"   class {CLASS_NAMES[c]:8s} n={m.sum():4d} mean {tot[m].mean():12.0f} max {tot[m].max():12.0f}" + (f" {extra(m)}" if extra else ""))
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
import lz4e_amd  # noqa
from lz4e_amd import corpus  # noqa

L = lz4e_amd.lib()
P = ctypes.c_void_p
L.lz4e_debug_compress_stamped.argtypes = [P] * 8 + [ctypes.c_uint32, ctypes.c_uint32, P, P]
L.lz4e_debug_compress_stamped.restype = ctypes.c_int

def run(name, data, bs, cls, label):
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
    dbg = torch.zeros(n * 16, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        r = L.lz4e_debug_compress_stamped(src.data_ptr(), offs.data_ptr(), lens.data_ptr(), tt.data_ptr(),
                                          dst.data_ptr(), doffs.data_ptr(), caps.data_ptr(), ret.data_ptr(),
                                          n, bs, s, dbg.data_ptr())
        assert r == 0
    torch.cuda.synchronize()
    d = dbg.cpu().numpy().reshape(n, 16).astype(np.float64)
    ph = ["setup", "slowwalk", "chainwalk", "tables", "commit", "emit"]
    srch = d[:, 6].astype(np.int64) & 0xFFFFFFFF
    seqs = d[:, 6].astype(np.int64) >> 32
    rem = d[:, 7].astype(np.int64) & 0xFFFFFFFF
    c3 = d[:, 7].astype(np.int64) >> 32
    fa, fev = (c3 & 0xFFFF), (c3 >> 16)
    tot = d[:, :6].sum(1)
    print(f"== {name} {label}: {n} blocks, mean cycles/block {tot.mean():.0f}, max {tot.max():.0f}; "
          f"seq/block {seqs.mean():.0f} searches {srch.mean():.0f} passes {rem.mean():.0f}; "
          f"cycles/seq {tot.sum() / max(1, seqs.sum()):.0f}; fast attempts {fa.mean():.0f} fast seqs {fev.mean():.0f}")
    for i, p in enumerate(ph):
        print(f"   {p:8s} {d[:, i].mean():12.0f}  ({100 * d[:, i].sum() / tot.sum():5.1f}%)")
    by_class(name, tot, n, lambda m: f"seq {seqs[m].mean():.0f} win {srch[m].mean():.0f} pass {rem[m].mean():.0f} att {fa[m].mean():.0f} fseq {fev[m].mean():.0f} " + " ".join(f"{ph[i]}={d[m, i].mean():.0f}" for i in range(6)))
    if name.startswith("silesia"):
        os.makedirs("gpurun_out", exist_ok=True)
        np.save(f"gpurun_out/stamps_{name}.npy", tot)  # per-block cycles (launch-order studies)
        cls = np.random.default_rng(0x5157).choice(6, size=n, p=[0.40, 0.15, 0.10, 0.10, 0.10, 0.15])
        top = np.argsort(-tot)[:12]
        print("   slowest blocks: " + ", ".join(f"{i}:{CLASS_NAMES[cls[i]]}:{tot[i] / 1e6:.2f}M" for i in top))
        for i in top[:4]:
            blk = data[i * bs:(i + 1) * bs]
            print(f"   block {i}: " + " ".join(f"{ph[k]}={d[i, k] / 1e6:.2f}M" for k in range(6)) +
                  f" seq {seqs[i]} win {srch[i]} pass {rem[i]} ratio {bs / max(1, int(ret[i])):.2f}"
                  f" head {bytes(blk[:24]).hex()}")

if __name__ == "__main__":
    mode = os.environ.get("LZ4E_COMPRESS_LDS_MAX", "default")
    if os.environ.get("STAMPS_U32"):  # the sg512 workload's class (byU32)
        run("silesia64k-u32", corpus.silesia_proxy(3234 * 65536, 0x5157), 65536, 3, f"lds_max={mode}")
    run("silesia64k", corpus.silesia_proxy(3234 * 65536, 0x5157), 65536, 1, f"lds_max={mode}")
    run("text64k", corpus.text_proxy(512 * 65536, 7), 65536, 1, f"lds_max={mode}")
    run("fio4k", corpus.fio_pattern(16384 * 4096), 4096, 1, f"lds_max={mode}")
