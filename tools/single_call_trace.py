"""Diagnostic: where a drop-in single call's time goes.  Runs N synchronous
LZ4E_compress_default / LZ4E_decompress_safe calls (configs[0]: 01.txt[0:4096],
one thread) and prints the host-side p50 of each; run it under
`rocprofv3 --kernel-trace --memory-copy-trace` and summarise the database with
tools/rocpd_stats.py to see the device-side share (kernels, copies) of a call.

usage: python tools/single_call_trace.py [calls]"""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import lz4e_amd  # noqa: E402
import oracle_ref  # noqa: E402
from lz4e_amd import BYU16, compress_bound, make_sg  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 300
data = open(os.path.join(REPO, "tests", "golden", "test_files", "01.txt"), "rb").read()[:4096]
n, cap = len(data), compress_bound(4096)
er, ef, _, _ = oracle_ref.compress(data, BYU16)
L = lz4e_amd.lib()
src = make_sg(data, [n])
dst = make_sg(b"", [4096, cap - 4096], capacity=cap)
wrk = (ctypes.c_uint8 * lz4e_amd.LZ4E_MEM_COMPRESS)()
fsrc = ctypes.create_string_buffer(ef, len(ef))
dout = ctypes.create_string_buffer(n + 16)
tc, td = [], []
for k in range(calls + 20):
    src.it.bi_size, src.it.bi_idx, src.it.bi_bvec_done = n, 0, 0
    dst.it.bi_size, dst.it.bi_idx, dst.it.bi_bvec_done = cap, 0, 0
    t0 = time.perf_counter()
    r = L.LZ4E_compress_default(src.bvecs, dst.bvecs, ctypes.byref(src.it), ctypes.byref(dst.it), wrk)
    t1 = time.perf_counter()
    d = L.LZ4E_decompress_safe(fsrc, dout, len(ef), n)
    t2 = time.perf_counter()
    assert r == er and d == n
    if k >= 20:
        tc.append(t1 - t0)
        td.append(t2 - t1)
print(f"single calls x{calls}: compress p50 {np.median(tc) * 1e6:.1f} us, decompress p50 {np.median(td) * 1e6:.1f} us",
      flush=True)
