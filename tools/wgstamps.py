"""Diagnostic: per-phase cycles of the workgroup decoder (stamped build), per
Silesia-proxy class, beside the kernel time of both decoders.

usage: python tools/wgstamps.py [blocks per class]"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
import lz4e_amd  # noqa: E402
from lz4e_amd import corpus  # noqa: E402

L = lz4e_amd.lib()
P = ctypes.c_void_p
L.lz4e_debug_decompress_stamped.argtypes = [P] * 7 + [ctypes.c_uint32, P, P, ctypes.c_uint32]
PH = ["stage+J1", "doubling", "tokens", "literals", "matches", "flush"]


def blocks(kind, n, bs=65536):
    rng = np.random.default_rng(5)
    jpg = np.frombuffer(corpus._jpeg(), np.uint8)
    gen = {"text": lambda: corpus.text_proxy(bs, int(rng.integers(1 << 30))),
           "ints": lambda: corpus._int_table(bs, rng), "records": lambda: corpus._records(bs, rng),
           "runs": lambda: corpus._runs(bs, rng),
           "random": lambda: rng.integers(0, 256, bs, dtype=np.uint8),
           "jpeg": lambda: jpg[(s := int(rng.integers(0, jpg.size - bs))):s + bs]}[kind]
    return np.concatenate([gen() for _ in range(n)])


def run(kind, data, bs=65536):
    dev = torch.device("cuda")
    n = data.size // bs
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
    dbg = torch.zeros(n * 8, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ms = {}
    for mc in (bs, 0):  # workgroup decoder, one-wave decoder
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            lz4e_amd.decompress_batch_dev(dst, doffs, ret, out, offs, lens, dret, max_cap=mc)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
            assert torch.equal(out[:n * bs], src), (kind, mc)
        ms[mc] = min(ts)
    assert L.lz4e_debug_decompress_stamped(dst.data_ptr(), doffs.data_ptr(), ret.data_ptr(),
                                           out.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                           dret.data_ptr(), n, s, dbg.data_ptr(), bs) == 0
    torch.cuda.synchronize()
    assert torch.equal(out[:n * bs], src)
    d = dbg.cpu().numpy().reshape(n, 8).astype(np.float64)
    tot = d[:, :6].sum(1)
    ratio = n * bs / ret.sum().item()
    print(f"== {kind:8s} {n} blocks ratio {ratio:.2f}: workgroup {ms[bs]:.3f} ms, one-wave {ms[0]:.3f} ms; "
          f"cycles/block mean {tot.mean():.0f} max {tot.max():.0f}; batches {d[:, 6].mean():.1f} "
          f"rounds {d[:, 7].mean():.1f}", flush=True)
    print("   " + "  ".join(f"{PH[i]} {d[:, i].mean():.0f}" for i in range(6)), flush=True)


if __name__ == "__main__":
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    for kind in ("text", "ints", "records", "runs", "random", "jpeg"):
        run(kind, blocks(kind, nb))
    run("silesia", corpus.silesia_proxy(1024 * 65536, 0x5157))
