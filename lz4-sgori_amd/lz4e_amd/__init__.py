"""lz4e_amd -- Python view of the MI355X-native LZ4E scatter-gather codec.

The product is the C-ABI library ``liblz4e_amd.so`` (include/lz4e.h): HIP
kernels for gfx950 plus a host shim.  This module only binds it with ctypes
so that tests and the benchmark can drive the same entry points a C caller
(the lz4e_bdev chunk layer, lz4e_bdev/lz4e_chunk.c:139-159) would use:

* :func:`compress_default`   -- ``LZ4E_compress_default`` (bio_vec in/out)
* :func:`decompress_safe`    -- ``LZ4E_decompress_safe``
* :func:`compress_sg_batch`  -- many SG requests, one launch
* :func:`compress_batch_dev` / :func:`decompress_batch_dev` -- device-resident
  batches on torch CUDA(HIP) tensors (the throughput path)

There is no CPU fallback: importing works without a GPU (so host-side
helpers and symbol checks can run anywhere), but every codec call fails
loudly (:class:`GpuUnavailable`) when the library cannot reach a gfx950.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

__all__ = [
    "PAGE_SIZE", "BIO_MAX_VECS", "LZ4E_MEM_COMPRESS", "LZ4E_MAX_INPUT_SIZE",
    "BYU16", "BYU32", "BYU64", "compress_bound", "BioVec", "BvecIter",
    "SgRequest", "SgList", "make_sg", "lib", "gpu_available", "table_type",
    "compress_default", "decompress_safe", "compress_sg_batch",
    "decompress_batch", "compress_batch_dev", "decompress_batch_dev",
    "GpuUnavailable", "LIB_PATH", "EXPORTED_SYMBOLS",
]

PAGE_SIZE = 4096
BIO_MAX_VECS = 256
LZ4E_MEM_COMPRESS = 17440
LZ4E_MAX_INPUT_SIZE = 0x7E000000
BYU16, BYU32, BYU64 = 1, 3, 7

LIB_PATH = os.environ.get("LZ4E_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblz4e_amd.so")

# Every function include/lz4e.h declares.
EXPORTED_SYMBOLS = (
    "LZ4E_compress_default", "LZ4E_decompress_safe", "lz4e_sg_table_type",
    "lz4e_last_error", "lz4e_gpu_available", "lz4e_compress_sg_batch",
    "lz4e_decompress_batch", "lz4e_compress_batch_dev", "lz4e_decompress_batch_dev",
    "lz4e_decompress_batch_dev2",
    "lz4e_chunk_write_batch", "lz4e_decompress_safe_sg", "lz4e_decompress_sg_batch",
    "LZ4E_compress_usingDict", "LZ4E_decompress_safe_usingDict", "lz4e_compress_sg_batch_dict",
    "lz4e_decompress_batch_dict", "lz4e_compress_batch_dev_dict", "lz4e_decompress_batch_dev_dict",
)


class GpuUnavailable(RuntimeError):
    """The library could not reach a gfx950 device (no fallback exists)."""


def compress_bound(n: int) -> int:
    """LZ4E_COMPRESSBOUND (lz4e/include/lz4e.h:25-28)."""
    return 0 if n > LZ4E_MAX_INPUT_SIZE else n + n // 255 + 16


class BioVec(ctypes.Structure):
    _fields_ = [("bv_page", ctypes.c_void_p), ("bv_len", ctypes.c_uint),
                ("bv_offset", ctypes.c_uint)]


class BvecIter(ctypes.Structure):
    _fields_ = [("bi_sector", ctypes.c_uint64), ("bi_size", ctypes.c_uint),
                ("bi_idx", ctypes.c_uint), ("bi_bvec_done", ctypes.c_uint)]

    def as_tuple(self) -> Tuple[int, int, int]:
        return (self.bi_size, self.bi_idx, self.bi_bvec_done)


class SgRequest(ctypes.Structure):
    _fields_ = [("src", ctypes.POINTER(BioVec)), ("dst", ctypes.POINTER(BioVec)),
                ("srcIter", ctypes.POINTER(BvecIter)), ("dstIter", ctypes.POINTER(BvecIter)),
                ("ret", ctypes.c_int)]


class ChunkRequest(ctypes.Structure):
    """struct lz4e_chunk_request (include/lz4e.h)."""
    _fields_ = [("src", ctypes.POINTER(BioVec)), ("srcIter", ctypes.POINTER(BvecIter)),
                ("data", ctypes.c_void_p), ("frame", ctypes.c_void_p), ("frame_cap", ctypes.c_int),
                ("comp_size", ctypes.c_int), ("status", ctypes.c_int)]


class ChunkStats(ctypes.Structure):
    """struct lz4e_chunk_stats (include/lz4e.h)."""
    _fields_ = [("reqs_total", ctypes.c_uint64), ("reqs_failed", ctypes.c_uint64),
                ("vec_count", ctypes.c_uint64), ("data_in_bytes", ctypes.c_uint64),
                ("frame_bytes", ctypes.c_uint64)]


EIO, ENOSPC = 5, 28

_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    """Load liblz4e_amd.so (raises ImportError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: build it with `make -C lz4-sgori_amd` "
                          "(or __graft_entry__.build())")
    # One HIP runtime per process: torch wheels bundle their own
    # libamdhip64.so.7 (same soname as /opt/rocm's).  Whichever loads first is
    # shared by both, and torch only initialises on its own copy, so when
    # torch is installed it is imported before the library is loaded.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    P, U32, I32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    L.LZ4E_compress_default.argtypes = [ctypes.POINTER(BioVec), ctypes.POINTER(BioVec),
                                        ctypes.POINTER(BvecIter), ctypes.POINTER(BvecIter), P]
    L.LZ4E_compress_default.restype = I32
    L.LZ4E_decompress_safe.argtypes = [P, P, I32, I32]
    L.LZ4E_decompress_safe.restype = I32
    L.lz4e_sg_table_type.argtypes = [ctypes.POINTER(BioVec), ctypes.POINTER(BvecIter)]
    L.lz4e_sg_table_type.restype = I32
    L.lz4e_last_error.argtypes = []
    L.lz4e_last_error.restype = ctypes.c_char_p
    L.lz4e_gpu_available.argtypes = []
    L.lz4e_gpu_available.restype = I32
    L.lz4e_compress_sg_batch.argtypes = [ctypes.POINTER(SgRequest), I32]
    L.lz4e_compress_sg_batch.restype = I32
    L.lz4e_decompress_batch.argtypes = [P, P, P, P, P, I32]
    L.lz4e_decompress_batch.restype = I32
    L.lz4e_compress_batch_dev.argtypes = [P, P, P, P, P, P, P, P, P, U32, U32, P]
    L.lz4e_compress_batch_dev.restype = I32
    L.lz4e_decompress_batch_dev.argtypes = [P, P, P, P, P, P, P, U32, P]
    L.lz4e_decompress_batch_dev.restype = I32
    L.lz4e_decompress_batch_dev2.argtypes = [P, P, P, P, P, P, P, U32, U32, P]
    L.lz4e_decompress_batch_dev2.restype = I32
    L.lz4e_chunk_write_batch.argtypes = [ctypes.POINTER(ChunkRequest), I32, ctypes.POINTER(ChunkStats)]
    L.lz4e_chunk_write_batch.restype = I32
    L.lz4e_decompress_safe_sg.argtypes = [P, ctypes.POINTER(BioVec), ctypes.POINTER(BvecIter), I32]
    L.lz4e_decompress_safe_sg.restype = I32
    L.lz4e_decompress_sg_batch.argtypes = [P, P, P, P, P, I32]
    L.lz4e_decompress_sg_batch.restype = I32
    L.LZ4E_compress_usingDict.argtypes = [ctypes.POINTER(BioVec), ctypes.POINTER(BioVec),
                                          ctypes.POINTER(BvecIter), ctypes.POINTER(BvecIter), P, P, I32]
    L.LZ4E_compress_usingDict.restype = I32
    L.LZ4E_decompress_safe_usingDict.argtypes = [P, P, I32, I32, P, I32]
    L.LZ4E_decompress_safe_usingDict.restype = I32
    L.lz4e_compress_sg_batch_dict.argtypes = [ctypes.POINTER(SgRequest), I32, P, P]
    L.lz4e_compress_sg_batch_dict.restype = I32
    L.lz4e_decompress_batch_dict.argtypes = [P, P, P, P, P, P, P, I32]
    L.lz4e_decompress_batch_dict.restype = I32
    L.lz4e_compress_batch_dev_dict.argtypes = [P, P, P, P, P, P, P, P, P, U32, U32, P, P]
    L.lz4e_compress_batch_dev_dict.restype = I32
    L.lz4e_decompress_batch_dev_dict.argtypes = [P, P, P, P, P, P, P, U32, U32, P, P]
    L.lz4e_decompress_batch_dev_dict.restype = I32
    _lib = L
    return L


def last_error() -> str:
    return lib().lz4e_last_error().decode()


def gpu_available() -> bool:
    return bool(lib().lz4e_gpu_available())


def _require_gpu() -> None:
    if not gpu_available():
        raise GpuUnavailable(last_error() or "lz4e: no usable gfx950 device")


# ---------------------------------------------------------------------------
# Scatter-gather buffers (userspace bio_vec lists backed by page-aligned memory)
# ---------------------------------------------------------------------------

@dataclass
class SgList:
    """A bio_vec list over page-aligned host memory plus an iterator into it."""
    backing: np.ndarray
    bvecs: ctypes.Array
    it: BvecIter
    seg_addr: List[int] = field(default_factory=list)

    @property
    def nseg(self) -> int:
        return len(self.bvecs)

    def read(self) -> bytes:
        """Bytes covered by the iterator (gathered)."""
        out = bytearray()
        size, idx, done = self.it.bi_size, self.it.bi_idx, self.it.bi_bvec_done
        while size:
            b = self.bvecs[idx]
            take = min(b.bv_len - done, size)
            out += ctypes.string_at(b.bv_page + b.bv_offset + done, take)
            size -= take
            done = 0
            idx += 1
        return bytes(out)

    def read_prefix(self, n: int) -> bytes:
        """First n bytes from the ORIGINAL start (segment order)."""
        out = bytearray()
        for b in self.bvecs:
            if len(out) >= n:
                break
            out += ctypes.string_at(b.bv_page + b.bv_offset, b.bv_len)
        return bytes(out[:n])


def make_sg(data: bytes, segments: Sequence[int], offsets: Optional[Sequence[int]] = None,
            start_done: int = 0, capacity: Optional[int] = None, shuffle_seed: Optional[int] = None,
            fill: int = 0) -> SgList:
    """Build a bio_vec list whose segments have the given lengths.

    Segment i lives at in-page offset offsets[i] (default 0) on its own run of
    pages (multi-page when offset + len > 4096); with ``shuffle_seed`` the page
    runs are placed in a shuffled order, so consecutive segments are not
    adjacent in memory.  ``data`` is written across the segments starting at
    byte ``start_done`` of segment 0; the iterator covers ``len(data)`` bytes
    (or ``capacity`` bytes for a destination list).
    """
    segments = list(segments)
    offsets = list(offsets) if offsets is not None else [0] * len(segments)
    runs = [max(1, -(-(o + ln) // PAGE_SIZE)) for o, ln in zip(offsets, segments)]
    order = list(range(len(segments)))
    if shuffle_seed is not None:
        rng = np.random.default_rng(shuffle_seed)
        rng.shuffle(order)
    start_page = [0] * len(segments)
    p = 0
    for i in order:
        start_page[i] = p
        p += runs[i]
    raw = np.full((p + 1) * PAGE_SIZE, fill, dtype=np.uint8)
    base = raw.ctypes.data
    aligned = (base + PAGE_SIZE - 1) // PAGE_SIZE * PAGE_SIZE
    bvecs = (BioVec * max(1, len(segments)))()
    addrs = []
    for i, (o, ln) in enumerate(zip(offsets, segments)):
        page = aligned + start_page[i] * PAGE_SIZE
        bvecs[i].bv_page = page
        bvecs[i].bv_len = ln
        bvecs[i].bv_offset = o
        addrs.append(page + o)
    # write data
    mv = memoryview(data)
    pos = 0
    for i, ln in enumerate(segments):
        lo = start_done if i == 0 else 0
        take = min(ln - lo, len(data) - pos)
        if take <= 0:
            break
        ctypes.memmove(addrs[i] + lo, bytes(mv[pos:pos + take]), take)
        pos += take
    size = capacity if capacity is not None else len(data)
    it = BvecIter(0, size, 0, start_done)
    return SgList(raw, bvecs, it, addrs)


def table_type(sg: SgList) -> int:
    """lz4e_sg_table_type: 1/3/7, or 0 for more than BIO_MAX_VECS segments."""
    return lib().lz4e_sg_table_type(sg.bvecs, ctypes.byref(sg.it))


# ---------------------------------------------------------------------------
# Reference entry points
# ---------------------------------------------------------------------------

def compress_default(src: SgList, dst: SgList, wrkmem: Optional[ctypes.Array] = None) -> int:
    """LZ4E_compress_default(src->bvecs, dst->bvecs, &src.it, &dst.it, wrkmem)."""
    _require_gpu()
    if wrkmem is None:
        wrkmem = (ctypes.c_uint8 * LZ4E_MEM_COMPRESS)()
    return lib().LZ4E_compress_default(src.bvecs, dst.bvecs, ctypes.byref(src.it),
                                       ctypes.byref(dst.it), wrkmem)


def decompress_safe(source: bytes, max_decompressed_size: int,
                    compressed_size: Optional[int] = None) -> Tuple[int, bytes]:
    """LZ4E_decompress_safe; returns (ret, dest[:max(ret, 0)])."""
    _require_gpu()
    csize = len(source) if compressed_size is None else compressed_size
    dst = ctypes.create_string_buffer(max(max_decompressed_size, 0) + 1)
    src = ctypes.create_string_buffer(bytes(source), max(len(source), 1))
    r = lib().LZ4E_decompress_safe(src, dst, csize, max_decompressed_size)
    return r, dst.raw[:max(r, 0)]


def compress_using_dict(src: SgList, dst: SgList, dictionary: bytes,
                        wrkmem: Optional[ctypes.Array] = None) -> int:
    """LZ4E_compress_usingDict (dictionary mode, include/lz4e.h)."""
    _require_gpu()
    if wrkmem is None:
        wrkmem = (ctypes.c_uint8 * LZ4E_MEM_COMPRESS)()
    d = ctypes.create_string_buffer(bytes(dictionary), max(len(dictionary), 1))
    return lib().LZ4E_compress_usingDict(src.bvecs, dst.bvecs, ctypes.byref(src.it),
                                         ctypes.byref(dst.it), wrkmem, d, len(dictionary))


def decompress_safe_using_dict(source: bytes, max_decompressed_size: int, dictionary: bytes,
                               compressed_size: Optional[int] = None) -> Tuple[int, bytes]:
    """LZ4E_decompress_safe_usingDict; returns (ret, dest[:max(ret, 0)])."""
    _require_gpu()
    csize = len(source) if compressed_size is None else compressed_size
    dst = ctypes.create_string_buffer(max(max_decompressed_size, 0) + 1)
    src = ctypes.create_string_buffer(bytes(source), max(len(source), 1))
    d = ctypes.create_string_buffer(bytes(dictionary), max(len(dictionary), 1))
    r = lib().LZ4E_decompress_safe_usingDict(src, dst, csize, max_decompressed_size, d,
                                             len(dictionary))
    return r, dst.raw[:max(r, 0)]


def decompress_batch_dict(frames: Sequence[bytes], caps: Sequence[int],
                          dicts: Sequence[bytes]) -> List[Tuple[int, bytes]]:
    """lz4e_decompress_batch_dict over host frames; returns (ret, bytes) per frame."""
    _require_gpu()
    n = len(frames)
    srcs = [ctypes.create_string_buffer(bytes(f), max(len(f), 1)) for f in frames]
    dsts = [ctypes.create_string_buffer(max(c, 0) + 1) for c in caps]
    dcs = [ctypes.create_string_buffer(bytes(d), max(len(d), 1)) for d in dicts]
    sp = (ctypes.c_void_p * n)(*[ctypes.addressof(s) for s in srcs])
    dp = (ctypes.c_void_p * n)(*[ctypes.addressof(d) for d in dsts])
    kp = (ctypes.c_void_p * n)(*[ctypes.addressof(d) for d in dcs])
    ks = (ctypes.c_int * n)(*[len(d) for d in dicts])
    cs = (ctypes.c_int * n)(*[len(f) for f in frames])
    cp = (ctypes.c_int * n)(*caps)
    rt = (ctypes.c_int * n)()
    if lib().lz4e_decompress_batch_dict(sp, cs, dp, cp, kp, ks, rt, n) < 0:
        raise GpuUnavailable(last_error())
    return [(rt[i], dsts[i].raw[:max(rt[i], 0)]) for i in range(n)]


def compress_sg_batch_dict(pairs: Sequence[Tuple[SgList, SgList]],
                           dicts: Sequence[bytes]) -> List[int]:
    """lz4e_compress_sg_batch_dict; returns each ret."""
    _require_gpu()
    n = len(pairs)
    reqs = (SgRequest * n)()
    for i, (s, d) in enumerate(pairs):
        reqs[i].src = s.bvecs
        reqs[i].dst = d.bvecs
        reqs[i].srcIter = ctypes.pointer(s.it)
        reqs[i].dstIter = ctypes.pointer(d.it)
    dcs = [ctypes.create_string_buffer(bytes(d), max(len(d), 1)) for d in dicts]
    kp = (ctypes.c_void_p * n)(*[ctypes.addressof(d) for d in dcs])
    ks = (ctypes.c_int * n)(*[len(d) for d in dicts])
    r = lib().lz4e_compress_sg_batch_dict(reqs, n, kp, ks)
    if r < 0:
        raise GpuUnavailable(last_error())
    return [reqs[i].ret for i in range(n)]


def compress_sg_batch(pairs: Sequence[Tuple[SgList, SgList]]) -> List[int]:
    """lz4e_compress_sg_batch over (src, dst) SG pairs; returns each ret."""
    _require_gpu()
    reqs = (SgRequest * len(pairs))()
    for i, (s, d) in enumerate(pairs):
        reqs[i].src = s.bvecs
        reqs[i].dst = d.bvecs
        reqs[i].srcIter = ctypes.pointer(s.it)
        reqs[i].dstIter = ctypes.pointer(d.it)
    r = lib().lz4e_compress_sg_batch(reqs, len(pairs))
    if r < 0:
        raise GpuUnavailable(last_error())
    return [reqs[i].ret for i in range(len(pairs))]


def decompress_batch(frames: Sequence[bytes], caps: Sequence[int]) -> List[Tuple[int, bytes]]:
    """lz4e_decompress_batch over host frames; returns (ret, bytes) per frame."""
    _require_gpu()
    n = len(frames)
    srcs = [ctypes.create_string_buffer(bytes(f), max(len(f), 1)) for f in frames]
    dsts = [ctypes.create_string_buffer(max(c, 0) + 1) for c in caps]
    sp = (ctypes.c_void_p * n)(*[ctypes.addressof(s) for s in srcs])
    dp = (ctypes.c_void_p * n)(*[ctypes.addressof(d) for d in dsts])
    cs = (ctypes.c_int * n)(*[len(f) for f in frames])
    cp = (ctypes.c_int * n)(*caps)
    rt = (ctypes.c_int * n)()
    if lib().lz4e_decompress_batch(sp, cs, dp, cp, rt, n) < 0:
        raise GpuUnavailable(last_error())
    return [(rt[i], dsts[i].raw[:max(rt[i], 0)]) for i in range(n)]


def decompress_safe_sg(source: bytes, dst: SgList, compressed_size: Optional[int] = None) -> int:
    """lz4e_decompress_safe_sg: decode into dst's segments from dst.it (capacity dst.it.bi_size)."""
    _require_gpu()
    csize = len(source) if compressed_size is None else compressed_size
    src = ctypes.create_string_buffer(bytes(source), max(len(source), 1))
    return lib().lz4e_decompress_safe_sg(src, dst.bvecs, ctypes.byref(dst.it), csize)


def decompress_sg_batch(frames: Sequence[bytes], dsts: Sequence[SgList]) -> List[int]:
    """lz4e_decompress_sg_batch; returns ret per frame (dst iterators advance on success)."""
    _require_gpu()
    n = len(frames)
    srcs = [ctypes.create_string_buffer(bytes(f), max(len(f), 1)) for f in frames]
    sp = (ctypes.c_void_p * n)(*[ctypes.addressof(s) for s in srcs])
    cs = (ctypes.c_int * n)(*[len(f) for f in frames])
    dp = (ctypes.c_void_p * n)(*[ctypes.addressof(d.bvecs) for d in dsts])
    ip = (ctypes.c_void_p * n)(*[ctypes.addressof(d.it) for d in dsts])
    rt = (ctypes.c_int * n)()
    if lib().lz4e_decompress_sg_batch(sp, cs, dp, ip, rt, n) < 0:
        raise GpuUnavailable(last_error())
    return list(rt)


def chunk_write_batch(srcs: Sequence[SgList], want_frames: bool = False,
                      stats: Optional[ChunkStats] = None):
    """lz4e_chunk_write_batch over WRITE bios given as SG lists.

    Returns (good, [(status, comp_size, data bytes, frame bytes or None)]),
    the chunk layer's result per request (lz4e_bdev/lz4e_req.c:144-213)."""
    _require_gpu()
    n = len(srcs)
    reqs = (ChunkRequest * max(1, n))()
    datas, frames = [], []
    for i, s in enumerate(srcs):
        size = s.it.bi_size
        d = ctypes.create_string_buffer(max(1, size))
        f = ctypes.create_string_buffer(max(1, compress_bound(size))) if want_frames else None
        datas.append(d)
        frames.append(f)
        reqs[i].src = s.bvecs
        reqs[i].srcIter = ctypes.pointer(s.it)
        reqs[i].data = ctypes.addressof(d)
        reqs[i].frame = ctypes.addressof(f) if f is not None else None
        reqs[i].frame_cap = compress_bound(size) if f is not None else 0
    good = lib().lz4e_chunk_write_batch(reqs, n, ctypes.byref(stats) if stats is not None else None)
    if good < 0:
        raise GpuUnavailable(last_error())
    out = []
    for i, s in enumerate(srcs):
        r = reqs[i]
        fr = frames[i].raw[:r.comp_size] if frames[i] is not None and r.status == 0 else None
        out.append((r.status, r.comp_size, datas[i].raw[:s.it.bi_size] if r.status == 0 else None, fr))
    return good, out


# ---------------------------------------------------------------------------
# Device-resident batches (torch tensors on the HIP device)
# ---------------------------------------------------------------------------

def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _check_dev(n: int, **tensors) -> None:
    """The kernels read raw pointers: every tensor must be contiguous, on one
    HIP device, of the element type the C ABI expects, and (descriptors) hold
    one entry per block -- a wrong dtype would be read as another width."""
    import torch
    want = {"src": torch.uint8, "dst": torch.uint8, "table_type": torch.uint8,
            "src_off": torch.int64, "dst_off": torch.int64, "src_len": torch.int32,
            "dst_cap": torch.int32, "ret": torch.int32, "aux": torch.int32}
    per_block = {"src_off": 1, "dst_off": 1, "src_len": 1, "dst_cap": 1, "ret": 1,
                 "table_type": 1, "aux": 2}
    dev = None
    for name, t in tensors.items():
        if t is None:
            continue
        if t.dtype != want[name]:
            raise TypeError(f"{name}: dtype {t.dtype}, expected {want[name]}")
        if not t.is_cuda:
            raise ValueError(f"{name}: not a device tensor")
        if not t.is_contiguous():
            raise ValueError(f"{name}: not contiguous")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError(f"{name}: on {t.device}, other tensors on {dev}")
        if name in per_block and t.numel() < per_block[name] * n:
            raise ValueError(f"{name}: {t.numel()} entries for {n} blocks")


def compress_batch_dev(src, src_off, src_len, table_type_, dst, dst_off, dst_cap, ret,
                       aux=None, max_len: Optional[int] = None, stream=None) -> None:
    """lz4e_compress_batch_dev on torch tensors (uint8 / int64 / int32 views).

    src/dst: uint8; src_off/dst_off: int64; src_len/dst_cap/ret: int32;
    table_type_: uint8; aux: int32 [2*nblocks] or None.  Launch only (async on
    ``stream``, default: torch's current stream).
    """
    import torch  # local: the package itself does not need torch
    n = int(src_len.numel())
    _check_dev(n, src=src, src_off=src_off, src_len=src_len, table_type=table_type_, dst=dst,
               dst_off=dst_off, dst_cap=dst_cap, ret=ret, aux=aux)
    if max_len is None:
        max_len = int(src_len.max().item()) if n else 0
    if stream is None:
        stream = torch.cuda.current_stream().cuda_stream
    r = lib().lz4e_compress_batch_dev(_ptr(src), _ptr(src_off), _ptr(src_len), _ptr(table_type_),
                                      _ptr(dst), _ptr(dst_off), _ptr(dst_cap), _ptr(ret), _ptr(aux),
                                      n, int(max_len), stream)
    if r != 0:
        raise RuntimeError("lz4e_compress_batch_dev: " + last_error())


def decompress_batch_dev(src, src_off, src_len, dst, dst_off, dst_cap, ret, stream=None,
                         max_cap: Optional[int] = None) -> None:
    """lz4e_decompress_batch_dev2 on torch tensors (launch only).

    ``max_cap`` bounds dst_cap (default: read from it, which synchronises);
    16 KiB and more selects the pipelined 4-wave decoder, smaller blocks
    decode on one wave each."""
    import torch
    n = int(src_len.numel())
    if max_cap is None:
        max_cap = int(dst_cap.max().item()) if n else 0
    # decompress descriptors: frame offsets int64, frame sizes / capacities / ret int32
    _check_dev(n, src=src, src_off=src_off, src_len=src_len, dst=dst, dst_off=dst_off,
               dst_cap=dst_cap, ret=ret)
    if stream is None:
        stream = torch.cuda.current_stream().cuda_stream
    r = lib().lz4e_decompress_batch_dev2(_ptr(src), _ptr(src_off), _ptr(src_len), _ptr(dst),
                                         _ptr(dst_off), _ptr(dst_cap), _ptr(ret), n,
                                         max(0, int(max_cap)), stream)
    if r != 0:
        raise RuntimeError("lz4e_decompress_batch_dev2: " + last_error())
