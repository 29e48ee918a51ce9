"""C-ABI checks that need no GPU: the library loads, exports every symbol
include/lz4e.h declares, its host-side SG logic matches the oracle, the
header's layouts match the reference's, and without a GPU the codec fails
loudly instead of falling back to a CPU path."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_ref
import lz4e_amd
from lz4e_amd import BYU16, BYU32, BYU64, make_sg

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "lz4e.h")


def _declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\**\s*\b((?:LZ4E|lz4e)_\w+)\s*\(", text, re.M)))


def test_library_exports_header_symbols(amd):
    names = _declared_functions()
    assert len(names) == len(lz4e_amd.EXPORTED_SYMBOLS)
    assert set(names) == set(lz4e_amd.EXPORTED_SYMBOLS)
    L = amd.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", lz4e_amd.LIB_PATH], capture_output=True, text=True)
    for n in names:
        assert hasattr(L, n)
        assert re.search(rf"\bT {n}$", out.stdout, re.M), n


def test_header_layouts(tmp_path):
    """sizeof(LZ4E_stream_t) == LZ4E_MEM_COMPRESS == 17440 (lz4e/include/lz4e.h:17-45)
    and the userspace bio_vec / bvec_iter match the ctypes mirrors."""
    src = tmp_path / "t.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "lz4e.h"\n'
        'int main(void){printf("%zu %zu %zu %zu %zu %zu %d\\n", sizeof(LZ4E_stream_t),'
        ' (size_t)LZ4E_MEM_COMPRESS, sizeof(struct bio_vec), sizeof(struct bvec_iter),'
        ' offsetof(struct bvec_iter, bi_size), offsetof(struct bio_vec, bv_offset),'
        ' LZ4E_COMPRESSBOUND(65536));\n'
        ' printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(struct lz4e_chunk_stats),'
        ' offsetof(struct lz4e_chunk_stats, vec_count), offsetof(struct lz4e_chunk_stats, data_in_bytes),'
        ' sizeof(struct lz4e_chunk_request), offsetof(struct lz4e_chunk_request, status),'
        ' sizeof(struct lz4e_sg_request)); return 0;}\n')
    exe = tmp_path / "t"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    vals = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    s_stream, memc, s_bv, s_it, o_size, o_off, bound = map(int, vals[:7])
    st_size, st_vec, st_data, rq_size, rq_status, sg_size = map(int, vals[7:])
    assert st_size == ctypes.sizeof(lz4e_amd.ChunkStats)
    assert st_vec == lz4e_amd.ChunkStats.vec_count.offset
    assert st_data == lz4e_amd.ChunkStats.data_in_bytes.offset
    assert rq_size == ctypes.sizeof(lz4e_amd.ChunkRequest)
    assert rq_status == lz4e_amd.ChunkRequest.status.offset
    assert sg_size == ctypes.sizeof(lz4e_amd.SgRequest)
    assert s_stream == memc == 17440
    assert s_bv == ctypes.sizeof(lz4e_amd.BioVec)
    assert s_it == ctypes.sizeof(lz4e_amd.BvecIter)
    assert o_size == lz4e_amd.BvecIter.bi_size.offset
    assert o_off == lz4e_amd.BioVec.bv_offset.offset
    assert bound == 65809 == lz4e_amd.compress_bound(65536)


@pytest.mark.parametrize("seed", range(20))
def test_table_type_matches_oracle(amd, seed):
    rng = np.random.default_rng(seed)
    k = int(rng.integers(1, 300))
    segs = [int(x) for x in rng.choice([1, 7, 512, 4096, 4097, 9000], size=k)]
    if seed == 3:
        segs = [(1 << 24) + 1, 10]
    n = sum(segs) - int(rng.integers(0, segs[-1]))
    start_done = int(rng.integers(0, segs[0]))
    n = max(0, n - start_done)
    src = make_sg(b"", segs, start_done=start_done, capacity=n) if seed != 3 else None
    if src is None:
        # a > 16 MiB segment without materialising it: fake pages are never read
        bv = (lz4e_amd.BioVec * 2)()
        bv[0].bv_len, bv[1].bv_len = segs
        it = lz4e_amd.BvecIter(0, sum(segs), 0, 0)
        got = amd.lib().lz4e_sg_table_type(bv, ctypes.byref(it))
        assert got == BYU64
        return
    assert amd.table_type(src) == oracle_ref.table_type(src)


def test_no_gpu_fails_loudly(amd):
    if amd.gpu_available():
        pytest.skip("a GPU is visible; the no-GPU contract is checked on CPU-only hosts")
    data = b"hello hello hello hello hello"
    src = make_sg(data, [len(data)])
    dst = make_sg(b"", [4096], capacity=128)
    wrk = (ctypes.c_uint8 * lz4e_amd.LZ4E_MEM_COMPRESS)()
    r = amd.lib().LZ4E_compress_default(src.bvecs, dst.bvecs, ctypes.byref(src.it), ctypes.byref(dst.it), wrk)
    assert r == 0
    assert "lz4e" in amd.last_error()
    assert src.it.bi_size == len(data)  # untouched on failure
    buf = ctypes.create_string_buffer(64)
    assert amd.lib().LZ4E_decompress_safe(b"\x10a", buf, 2, 64) < 0
    with pytest.raises(amd.GpuUnavailable):
        amd.compress_default(src, dst)


def test_chunk_write_batch_no_gpu(amd):
    """Without a GPU the chunk pipeline reports -1 and marks every request -EIO."""
    if amd.gpu_available():
        pytest.skip("a GPU is visible")
    data = b"abcd" * 100
    src = make_sg(data, [len(data)])
    reqs = (lz4e_amd.ChunkRequest * 1)()
    buf = ctypes.create_string_buffer(len(data))
    reqs[0].src = src.bvecs
    reqs[0].srcIter = ctypes.pointer(src.it)
    reqs[0].data = ctypes.addressof(buf)
    st = lz4e_amd.ChunkStats()
    assert amd.lib().lz4e_chunk_write_batch(reqs, 1, ctypes.byref(st)) == -1
    assert reqs[0].status == -lz4e_amd.EIO and reqs[0].comp_size == 0
    with pytest.raises(amd.GpuUnavailable):
        amd.chunk_write_batch([src])


def test_coalescer_unwinds_a_throwing_batch(amd):
    """The single-call coalescer (csrc/lz4e_host.hip, Coalescer::submit): when
    a batch's run throws (here an injected fault, lz4e_debug_coalescer_fault;
    in the field std::bad_alloc from its staging), every caller of that batch
    returns -- a failure with the reason in lz4e_last_error -- and the next
    calls are served, on a GPU box and off it."""
    import threading

    L = amd.lib()
    L.lz4e_debug_coalescer_fault.argtypes = [ctypes.c_int]
    L.lz4e_debug_coalescer_fault.restype = ctypes.c_int
    L.lz4e_last_error.restype = ctypes.c_char_p
    os.environ.pop("LZ4E_TEST_FAULTS", None)
    assert L.lz4e_debug_coalescer_fault(1) == -1  # refused unless armed by the environment
    os.environ["LZ4E_TEST_FAULTS"] = "1"
    assert L.lz4e_debug_coalescer_fault(1 << 20) == 0
    results = []

    def caller(k):
        for _ in range(4):
            buf = ctypes.create_string_buffer(64)
            r = L.LZ4E_decompress_safe(b"\x10a" * (1 + k % 3), buf, 2, 64)
            results.append((r, L.lz4e_last_error().decode()))
            data = b"abc" * 40
            src = make_sg(data, [len(data)])
            dst = make_sg(b"", [4096], capacity=256)
            wrk = (ctypes.c_uint8 * lz4e_amd.LZ4E_MEM_COMPRESS)()
            rc = L.LZ4E_compress_default(src.bvecs, dst.bvecs, ctypes.byref(src.it), ctypes.byref(dst.it), wrk)
            results.append((rc - 1 if rc == 0 else rc, L.lz4e_last_error().decode()))

    try:
        ts = [threading.Thread(target=caller, args=(k,)) for k in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=60)
        assert not any(t.is_alive() for t in ts), "a caller of a throwing batch never returned"
    finally:
        L.lz4e_debug_coalescer_fault(0)
        os.environ.pop("LZ4E_TEST_FAULTS", None)
    assert len(results) == 64
    assert all(r < 0 and "injected fault" in e for r, e in results), results[:4]
    # the coalescer still serves calls
    buf = ctypes.create_string_buffer(64)
    r = L.LZ4E_decompress_safe(b"\x10a", buf, 2, 64)
    if amd.gpu_available():
        assert r == 1 and buf.raw[:1] == b"a"
    else:
        assert r < 0 and "injected" not in L.lz4e_last_error().decode()
