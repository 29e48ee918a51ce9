"""Diagnostic: the two decoders side by side per Silesia-proxy class -- kernel
time of the one-wave decoder and of the pipelined 4-wave decoder (outputs
checked equal to the input), plus the pipelined decoder's per-block cycle
counters (stamped build): parser parse / wait, copier work, copier waits for
records, far loads, batch j-1 and the store flag (summed over copiers).

usage: python tools/decab.py [blocks per class]"""
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
L.lz4e_debug_decompress_stamped.argtypes = [P] * 7 + [ctypes.c_uint32, P, P, ctypes.c_uint32,
                                                       ctypes.c_uint32]
PH = ["parse", "p_wait", "c_other", "c_rec", "c_far", "c_prev", "c_store", "batches", "c_loads",
      "c_rounds", "c_gather", "c_spass", "c_vm", "n_rounds", "n_int", "c_ptrs",
      "p_win", "p_comp", "p_follow", "p_fields", "blk_cycles", "blk_ticks"]
NS = len(PH)
WAVE, PIPE = 1, 2


def blocks(kind, n, bs):
    rng = np.random.default_rng(5)
    jpg = np.frombuffer(corpus._jpeg(), np.uint8)
    gen = {"text": lambda: corpus.text_proxy(bs, int(rng.integers(1 << 30))),
           "ints": lambda: corpus._int_table(bs, rng), "records": lambda: corpus._records(bs, rng),
           "runs": lambda: corpus._runs(bs, rng),
           "random": lambda: rng.integers(0, 256, bs, dtype=np.uint8),
           "jpeg": lambda: jpg[(s := int(rng.integers(0, jpg.size - bs))):s + bs]}[kind]
    return np.concatenate([gen() for _ in range(n)])


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
    lz4e_amd.compress_batch_dev(src, offs, lens, tt, dst, doffs, caps, ret)
    out = torch.zeros(n * bs + 64, dtype=torch.uint8, device=dev)
    dret = torch.zeros(n, dtype=torch.int32, device=dev)
    dbg = torch.zeros(n * NS, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def launch(mode, d=None):
        assert L.lz4e_debug_decompress_stamped(dst.data_ptr(), doffs.data_ptr(), ret.data_ptr(),
                                               out.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                               dret.data_ptr(), n, s, d, bs, mode) == 0

    ms = {}
    for mode in (WAVE, PIPE):
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
    launch(PIPE, dbg.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(out[:n * bs], src)
    d = dbg.cpu().numpy().reshape(n, NS).astype(np.float64)
    ratio = n * bs / ret.sum().item()
    print(f"== {kind:8s} {n} x {bs} ratio {ratio:.2f}: one-wave {ms[WAVE]:.3f} ms, pipelined "
          f"{ms[PIPE]:.3f} ms ({ms[WAVE] / ms[PIPE]:.2f}x)", flush=True)
    nb = max(1.0, d[:, 7].sum())
    print("   per batch: " + "  ".join(f"{PH[i]} {d[:, i].sum() / nb:.0f}" for i in range(NS - 2) if i != 7)
          + f"  (batches/block {d[:, 7].mean():.0f}, max {d[:, 7].max():.0f}; block cycles mean "
          f"{d[:, NS - 2].mean() / 1e3:.0f} k, max {d[:, NS - 2].max() / 1e3:.0f} k)", flush=True)


if __name__ == "__main__":
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    for kind in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("text", "ints", "records", "runs", "random", "jpeg")):
        run(kind, blocks(kind, nb, 65536))
    sil = corpus.silesia_proxy(3234 * 65536, 0x5157)
    run("silesia", sil)
    if os.environ.get("DECAB_ORDER"):
        # the same blocks, heaviest classes first (ints, records, text, runs, jpeg, random)
        cls = np.random.default_rng(0x5157).choice(6, size=3234, p=[0.40, 0.15, 0.10, 0.10, 0.10, 0.15])
        rank = np.array([2, 0, 3, 5, 4, 1])[cls]
        order = np.argsort(rank, kind="stable")
        run("sil-heavy1st", sil.reshape(3234, 65536)[order].reshape(-1))
        run("sil-light1st", sil.reshape(3234, 65536)[order[::-1]].reshape(-1))
    if os.environ.get("DECAB_ALL"):
        run("text256k", corpus.text_proxy(953 * 262144, 7), 262144, 3)
        run("fio4k", corpus.fio_pattern(65536 * 4096), 4096)
