"""Diagnostic: where a lone drop-in call's kernel time goes.

For configs[0] (01.txt[0:4096], byU16) it measures, on the GPU box:
  * the drop-in calls' host p50 (LZ4E_compress_default / LZ4E_decompress_safe,
    one thread), as tools/single_call_trace.py;
  * the same block compressed and decoded alone through the stamped kernels,
    each after the chip sat idle for 0.5 s ("cold") and right after a busy
    second of full-batch work ("warm"): the kernel's shader cycles and its
    s_memrealtime ticks (100 MHz) from inside the kernel, hence the clock the
    lone wave ran at and its wall time;
  * the same block's cycles when it is one of 2 560 copies in one launch
    (the chip full, as in a batch);
  * the clock probe's reading right after the idle wait (one wave, ~16 k
    cycles of dependent VALU work).
A lone call's kernel time = (its cycles) / (its clock); the cycles split into
the serial chain (the in-batch cycles, warm) and whatever a cold start adds.

usage: python tools/single_call_clock.py [reps]"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import lz4e_amd  # noqa: E402
import oracle_ref  # noqa: E402
from lz4e_amd import BYU16, compress_bound, make_sg  # noqa: E402

L = lz4e_amd.lib()
P = ctypes.c_void_p
L.lz4e_debug_compress_stamped.argtypes = [P] * 8 + [ctypes.c_uint32, ctypes.c_uint32, P, P]
L.lz4e_debug_decompress_stamped.argtypes = [P] * 7 + [ctypes.c_uint32, P, P, ctypes.c_uint32, ctypes.c_uint32]
L.lz4e_debug_clock_probe.argtypes = [P, P, ctypes.c_uint32]
CW = 16          # kCompressStampWords
PIPE_SLOTS = 22  # kStSlots of the pipelined decoder (kStT = 20, kStR = 21)

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda")
data = open(os.path.join(REPO, "tests", "golden", "test_files", "01.txt"), "rb").read()[:4096]
n, cap = len(data), compress_bound(4096)
er, ef, _, _ = oracle_ref.compress(data, BYU16)
stream = torch.cuda.Stream()
s = stream.cuda_stream


def mk(nb):
    src = torch.from_numpy(np.frombuffer(data * nb, np.uint8).copy()).to(dev)
    off = torch.arange(nb, dtype=torch.int64, device=dev) * n
    ln = torch.full((nb,), n, dtype=torch.int32, device=dev)
    tt = torch.full((nb,), BYU16, dtype=torch.uint8, device=dev)
    slot = (cap + 79) // 16 * 16
    doff = torch.arange(nb, dtype=torch.int64, device=dev) * slot
    dcap = torch.full((nb,), cap, dtype=torch.int32, device=dev)
    dst = torch.zeros(nb * slot + 64, dtype=torch.uint8, device=dev)
    ret = torch.zeros(nb, dtype=torch.int32, device=dev)
    return dict(nb=nb, src=src, off=off, ln=ln, tt=tt, doff=doff, dcap=dcap, dst=dst, ret=ret,
                out=torch.zeros(nb * n + 64, dtype=torch.uint8, device=dev),
                dret=torch.zeros(nb, dtype=torch.int32, device=dev))


def compress(b, dbg=None):
    with torch.cuda.stream(stream):
        rc = L.lz4e_debug_compress_stamped(b["src"].data_ptr(), b["off"].data_ptr(), b["ln"].data_ptr(),
                                           b["tt"].data_ptr(), b["dst"].data_ptr(), b["doff"].data_ptr(),
                                           b["dcap"].data_ptr(), b["ret"].data_ptr(), b["nb"], n, s,
                                           dbg.data_ptr() if dbg is not None else None)
    assert rc == 0
    stream.synchronize()


def decompress(b, mode, dbg=None):
    rc = L.lz4e_debug_decompress_stamped(b["dst"].data_ptr(), b["doff"].data_ptr(), b["ret"].data_ptr(),
                                         b["out"].data_ptr(), b["off"].data_ptr(), b["ln"].data_ptr(),
                                         b["dret"].data_ptr(), b["nb"], s,
                                         dbg.data_ptr() if dbg is not None else None, n, mode)
    assert rc == 0
    stream.synchronize()


def busy(big, secs=1.0):
    t = time.time()
    while time.time() - t < secs:
        compress(big)


def probe():
    out = torch.zeros(3, dtype=torch.int64, device=dev)
    assert L.lz4e_debug_clock_probe(s, out.data_ptr(), 1 << 12) == 0
    stream.synchronize()
    mt, rt = (int(v) for v in out[:2].cpu())
    return mt / rt * 0.1 if rt else None


one, big = mk(1), mk(2560)
compress(one)
assert int(one["ret"][0]) == er and one["dst"][:er].cpu().numpy().tobytes() == ef
res = {"block": "01.txt[0:4096] byU16", "frame": er}

# drop-in calls (host p50), as tools/single_call_trace.py
src = make_sg(data, [n])
dsg = make_sg(b"", [4096, cap - 4096], capacity=cap)
wrk = (ctypes.c_uint8 * lz4e_amd.LZ4E_MEM_COMPRESS)()
fsrc = ctypes.create_string_buffer(ef, len(ef))
dout = ctypes.create_string_buffer(n + 16)
tc, td = [], []
for k in range(220):
    src.it.bi_size, src.it.bi_idx, src.it.bi_bvec_done = n, 0, 0
    dsg.it.bi_size, dsg.it.bi_idx, dsg.it.bi_bvec_done = cap, 0, 0
    t0 = time.perf_counter()
    r = L.LZ4E_compress_default(src.bvecs, dsg.bvecs, ctypes.byref(src.it), ctypes.byref(dsg.it), wrk)
    t1 = time.perf_counter()
    d = L.LZ4E_decompress_safe(fsrc, dout, len(ef), n)
    t2 = time.perf_counter()
    assert r == er and d == n
    if k >= 20:
        tc.append(t1 - t0)
        td.append(t2 - t1)
res["dropin_p50_us"] = {"compress": round(float(np.median(tc)) * 1e6, 1),
                        "decompress": round(float(np.median(td)) * 1e6, 1)}


def lone(kind, state):
    rows = []
    for _ in range(reps):
        if state == "cold":
            time.sleep(0.5)
        else:
            busy(big, 1.0)
        if kind == "compress":
            dbg = torch.zeros(CW, dtype=torch.int64, device=dev)
            compress(one, dbg)
            d = dbg.cpu().numpy()
            cyc, tick = int(d[8]), int(d[9])
        else:
            mode = {"decode_pipe": 2, "decode_wave": 1, "decode_lds": 6}[kind]
            w = PIPE_SLOTS if mode == 2 else 8
            dbg = torch.zeros(w, dtype=torch.int64, device=dev)
            decompress(one, mode, dbg)
            assert int(one["dret"][0]) == n
            d = dbg.cpu().numpy()
            cyc, tick = (int(d[20]), int(d[21])) if mode == 2 else (int(d[6]), int(d[7]))
        rows.append((cyc, tick))
    cyc = float(np.median([r[0] for r in rows]))
    tick = float(np.median([r[1] for r in rows]))
    return {"cycles": int(cyc), "us": round(tick / 100.0, 2), "clock_ghz": round(cyc / tick * 0.1, 3) if tick else None,
            "runs": [[c, t] for c, t in rows]}


time.sleep(0.5)
res["probe_clock_after_idle_ghz"] = probe()
busy(big, 1.0)
res["probe_clock_after_busy_ghz"] = probe()
for kind in ("compress", "decode_pipe", "decode_wave", "decode_lds"):
    res[kind] = {st: lone(kind, st) for st in ("cold", "warm")}
# in-batch cycles of the same block (2 560 copies: the chip full)
dbg = torch.zeros(big["nb"] * CW, dtype=torch.int64, device=dev)
busy(big, 0.5)
compress(big, dbg)
d = dbg.view(big["nb"], CW).cpu().numpy()
res["compress_in_batch"] = {"blocks": big["nb"], "cycles_median": int(np.median(d[:, 8])),
                            "cycles_max": int(d[:, 8].max()),
                            "clock_ghz_median": round(float(np.median(d[:, 8] / np.maximum(d[:, 9], 1) * 0.1)), 3)}
dbg = torch.zeros(big["nb"] * PIPE_SLOTS, dtype=torch.int64, device=dev)
decompress(big, 2, dbg)
d = dbg.view(big["nb"], PIPE_SLOTS).cpu().numpy()
res["decode_pipe_in_batch"] = {"blocks": big["nb"], "cycles_median": int(np.median(d[:, 20])),
                               "clock_ghz_median": round(float(np.median(d[:, 20] / np.maximum(d[:, 21], 1) * 0.1)), 3)}
print(json.dumps(res, indent=1))
