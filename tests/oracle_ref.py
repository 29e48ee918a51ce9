"""ctypes binding of oracle/liblz4e_oracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference path (see
oracle/lz4e_oracle.h); tests use it as the checker, bench.py as the timed
CPU baseline.  The product never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liblz4e_oracle.so")

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_SO):
        build()
    import lz4e_amd  # for the BioVec / BvecIter ctypes layouts only
    L = ctypes.CDLL(ORACLE_SO)
    P, U32, I32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    L.oracle_table_type.argtypes = [ctypes.POINTER(lz4e_amd.BioVec), ctypes.POINTER(lz4e_amd.BvecIter)]
    L.oracle_table_type.restype = I32
    L.oracle_compress_linear.argtypes = [P, U32, I32, P, U32, ctypes.POINTER(U32), ctypes.POINTER(U32)]
    L.oracle_compress_linear.restype = I32
    L.oracle_compress_sg.argtypes = [ctypes.POINTER(lz4e_amd.BioVec), ctypes.POINTER(lz4e_amd.BioVec),
                                     ctypes.POINTER(lz4e_amd.BvecIter), ctypes.POINTER(lz4e_amd.BvecIter), P]
    L.oracle_compress_sg.restype = I32
    L.oracle_decompress_safe.argtypes = [P, P, I32, I32]
    L.oracle_decompress_safe.restype = I32
    L.oracle_compress_linear_batch.argtypes = [P, P, P, P, P, P, P, P, U32, I32]
    L.oracle_compress_linear_batch.restype = None
    L.oracle_compress_sg_batch.argtypes = [P, P, P, U32, P, P, P, P, U32, I32]
    L.oracle_compress_sg_batch.restype = None
    L.oracle_decompress_batch.argtypes = [P, P, P, P, P, P, P, U32, I32]
    L.oracle_decompress_batch.restype = None
    L.oracle_compress_dict.argtypes = [P, U32, P, U32, P, U32]
    L.oracle_compress_dict.restype = I32
    L.oracle_decompress_dict.argtypes = [P, P, I32, I32, P, I32]
    L.oracle_decompress_dict.restype = I32
    _lib = L
    return L


def compress(data: bytes, table_type: int, cap=None):
    """-> (ret, frame, final_src, last_run)."""
    L = load()
    n = len(data)
    cap = n + n // 255 + 16 if cap is None else cap
    out = ctypes.create_string_buffer(max(cap, 1) + 64)
    fs, lr = ctypes.c_uint32(), ctypes.c_uint32()
    src = ctypes.create_string_buffer(bytes(data), max(n, 1))
    r = L.oracle_compress_linear(src, n, table_type, out, cap, ctypes.byref(fs), ctypes.byref(lr))
    return r, out.raw[:max(r, 0)], fs.value, lr.value


def decompress(frame: bytes, cap: int, csize=None):
    """-> (ret, bytes[:max(ret,0)])."""
    L = load()
    csize = len(frame) if csize is None else csize
    out = ctypes.create_string_buffer(max(cap, 0) + 64)
    src = ctypes.create_string_buffer(bytes(frame), max(len(frame), 1))
    r = L.oracle_decompress_safe(src, out, csize, cap)
    return r, out.raw[:max(r, 0)]


def compress_dict(data: bytes, dictionary: bytes, cap=None):
    """Dictionary mode (LZ4E extension, parity unpinned) -> (ret, frame)."""
    L = load()
    n = len(data)
    cap = n + n // 255 + 16 if cap is None else cap
    out = ctypes.create_string_buffer(max(cap, 1) + 64)
    src = ctypes.create_string_buffer(bytes(data), max(n, 1))
    dct = ctypes.create_string_buffer(bytes(dictionary), max(len(dictionary), 1))
    r = L.oracle_compress_dict(src, n, dct, len(dictionary), out, cap)
    return r, out.raw[:max(r, 0)]


def decompress_dict(frame: bytes, cap: int, dictionary: bytes, csize=None):
    """-> (ret, bytes[:max(ret,0)]) decoding with a dictionary."""
    L = load()
    csize = len(frame) if csize is None else csize
    out = ctypes.create_string_buffer(max(cap, 0) + 64)
    src = ctypes.create_string_buffer(bytes(frame), max(len(frame), 1))
    dct = ctypes.create_string_buffer(bytes(dictionary), max(len(dictionary), 1))
    r = L.oracle_decompress_dict(src, out, csize, cap, dct, len(dictionary))
    return r, out.raw[:max(r, 0)]


def compress_sg(src_sg, dst_sg):
    L = load()
    wrk = (ctypes.c_uint8 * 17440)()
    return L.oracle_compress_sg(src_sg.bvecs, dst_sg.bvecs, ctypes.byref(src_sg.it),
                                ctypes.byref(dst_sg.it), wrk)


def table_type(sg) -> int:
    return load().oracle_table_type(sg.bvecs, ctypes.byref(sg.it))


def compress_blocks(data: np.ndarray, offs, lens, ttypes, threads: int = 1):
    """Batch compress of blocks of a flat uint8 array -> (ret int32[], frames list)."""
    L = load()
    n = len(lens)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    tt = np.ascontiguousarray(ttypes, dtype=np.uint8)
    caps = (lens.astype(np.uint64) + lens // 255 + 16).astype(np.uint32)
    ooff = np.zeros(n, dtype=np.uint64)
    ooff[1:] = np.cumsum(caps.astype(np.uint64) + 64)[:-1]
    out = np.zeros(int(ooff[-1] + caps[-1] + 64) if n else 1, dtype=np.uint8)
    ret = np.zeros(n, dtype=np.int32)
    data = np.ascontiguousarray(data)
    L.oracle_compress_linear_batch(data.ctypes.data, offs.ctypes.data, lens.ctypes.data, tt.ctypes.data,
                                   out.ctypes.data, ooff.ctypes.data, caps.ctypes.data, ret.ctypes.data,
                                   n, threads)
    frames = [out[int(ooff[i]):int(ooff[i]) + max(int(ret[i]), 0)].tobytes() for i in range(n)]
    return ret, frames
