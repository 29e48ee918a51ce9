"""Diagnostic: the chunked decoder's stamped build (mode 4, per-block cycle
and event counters, CkSt in csrc/lz4e_decompress.hip) per corpus class:
where a block's cycles go -- token walks, batch fields, copies (and the part
before the readiness rounds), exact-path steps, flushes / slides -- and the
events behind them (walk verification rounds per chunk, sequences per batch,
readiness rounds and pointer-jumping fallbacks per batch).

usage: python tools/ckstamps.py [blocks per class]"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import lz4e_amd  # noqa: E402
from lz4e_amd import corpus  # noqa: E402
from decmodes import class_blocks  # noqa: E402

L = lz4e_amd.lib()
P = ctypes.c_void_p
L.lz4e_debug_decompress_stamped.argtypes = [P] * 7 + [ctypes.c_uint32, P, P, ctypes.c_uint32,
                                                       ctypes.c_uint32]
NAMES = ["parse", "p_rounds", "chunks", "fields", "copy", "batches", "seqs", "exact", "n_exact",
         "flush_slide", "rounds", "pj", "total", "copy_pre"]
NS = 20


def run(name, data, bs, cls):
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
    lz4e_amd.compress_batch_dev(src, offs, lens, tt, dst, doffs, caps, ret)
    out = torch.zeros(n * bs + 64, dtype=torch.uint8, device=dev)
    dret = torch.zeros(n, dtype=torch.int32, device=dev)
    dbg = torch.zeros(n * NS, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    assert L.lz4e_debug_decompress_stamped(dst.data_ptr(), doffs.data_ptr(), ret.data_ptr(), out.data_ptr(),
                                           offs.data_ptr(), lens.data_ptr(), dret.data_ptr(), n, s,
                                           dbg.data_ptr(), bs, 4) == 0
    torch.cuda.synchronize()
    assert torch.equal(out[:n * bs], src) and bool((dret == lens).all().item()), name
    d = dbg.cpu().numpy().reshape(n, NS).astype(np.float64)
    S = {k: d[:, i].mean() for i, k in enumerate(NAMES)}
    nb, nc = max(S["batches"], 1e-9), max(S["chunks"], 1e-9)
    print(f"== {name:10s} {n} x {bs}: cycles/block {S['total']:.0f} = parse {S['parse'] / S['total']:.0%} "
          f"fields {S['fields'] / S['total']:.0%} copy {S['copy'] / S['total']:.0%} (pre-rounds "
          f"{S['copy_pre'] / S['total']:.0%}) exact {S['exact'] / S['total']:.0%} flush/slide "
          f"{S['flush_slide'] / S['total']:.0%}", flush=True)
    print(f"   per block: chunks {nc:.1f}, batches {nb:.1f}, exact steps {S['n_exact']:.1f}; per chunk: "
          f"walk rounds {S['p_rounds'] / nc:.2f}, cycles {S['parse'] / nc:.0f}; per batch: seqs "
          f"{S['seqs'] / nb:.1f}, rounds {S['rounds'] / nb:.2f}, pj {S['pj'] / nb:.2f}, fields "
          f"{S['fields'] / nb:.0f} cyc, copy {S['copy'] / nb:.0f} cyc (pre {S['copy_pre'] / nb:.0f}); per "
          f"exact step {S['exact'] / max(S['n_exact'], 1e-9):.0f} cyc", flush=True)


if __name__ == "__main__":
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    for kind in ("text", "ints", "records", "runs", "random", "jpeg"):
        run(kind, class_blocks(kind, nb, 65536), 65536, 1)
    run("text256k", corpus.text_proxy(256 * 262144, 0x7E57), 262144, 3)
    run("fio4k", corpus.fio_pattern(16384 * 4096), 4096, 1)
