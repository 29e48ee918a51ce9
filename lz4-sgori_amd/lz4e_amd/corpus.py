"""Seeded synthetic corpora for the LZ4E benchmarks.

Silesia and enwik9 are not available offline, so the benchmark uses proxies
of the same shape; every generator is deterministic in its seed.

* :func:`silesia_proxy` -- mixed-class blocks (word-level text drawn from the
  reference's own lorem test files, little-endian integer tables, runs and
  zeros, PRNG bytes, slices of the reference's 03.jpg, structured records);
  LZ4 ratio about 2.
* :func:`fio_pattern`   -- fio ``buffer_compress_percentage=50`` with
  ``buffer_compress_chunk=512``: per 512 B, 256 random bytes then 256 zeros.
* :func:`text_proxy`    -- word-level text only (the enwik9 proxy).
"""
from __future__ import annotations

import os
import re
from functools import lru_cache

import numpy as np

_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests", "golden",
                       "test_files")


@lru_cache(maxsize=1)
def _words() -> tuple:
    text = b""
    for name in ("01.txt", "02.txt"):
        p = os.path.join(_GOLDEN, name)
        if os.path.exists(p):
            with open(p, "rb") as f:
                text += f.read() + b" "
    if not text:
        text = b"lorem ipsum dolor sit amet consectetur adipiscing elit sed do eiusmod tempor"
    toks = re.findall(rb"[A-Za-z]+[,.]?", text)
    vocab, counts = np.unique(np.array(toks, dtype=object), return_counts=True)
    return tuple(vocab), counts / counts.sum()


@lru_cache(maxsize=1)
def _jpeg() -> bytes:
    p = os.path.join(_GOLDEN, "03.jpg")
    if os.path.exists(p):
        with open(p, "rb") as f:
            return f.read()
    return bytes(np.random.default_rng(3).integers(0, 256, 275147, dtype=np.uint8))


def _choice(rng, n: int, prob) -> np.ndarray:
    """rng.choice(len(prob), size=n, p=prob), bit for bit, without its slow
    binary search: the same uniforms (drawn in pieces: one stream), mapped
    through a 2^16-bucket table of the CDF; only uniforms in a bucket that
    straddles a CDF step take the search."""
    cdf = np.cumsum(prob)
    cdf /= cdf[-1]
    K = 1 << 16
    edges = np.arange(K + 1, dtype=np.float64) / K
    ss = cdf.searchsorted(edges, side="right")
    lo, hi = ss[:-1], ss[1:]
    out = np.empty(n, dtype=np.int64)
    for a in range(0, n, 1 << 24):
        u = rng.random(min(1 << 24, n - a))
        b = (u * K).astype(np.int64)
        r = lo[b]
        amb = lo[b] != hi[b]
        r[amb] = cdf.searchsorted(u[amb], side="right")
        out[a:a + u.size] = r
    return out


def text_proxy(nbytes: int, seed: int = 0x7E57) -> np.ndarray:
    """Word-level text from the lorem vocabulary, with sentence/line breaks."""
    rng = np.random.default_rng(seed)
    vocab, prob = _words()
    lens = np.array([len(w) + 1 for w in vocab])
    mean = float((lens * prob).sum())
    nwords = int(nbytes / mean * 1.05) + 16
    idx = _choice(rng, nwords, prob)
    # vocabulary bytes with a trailing separator; every ~12th separator a newline
    flat = np.frombuffer(b"".join(w + b" " for w in vocab), dtype=np.uint8)
    start = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    wl = lens[idx]
    out = np.empty(int(wl.sum()), dtype=np.uint8)
    # gather the words in pieces (bounded temporaries), then the newlines:
    # the same bytes and random stream as concatenating word by word
    step, o = 1 << 22, 0
    for a in range(0, nwords, step):
        ii, ll = idx[a:a + step], wl[a:a + step]
        tot = int(ll.sum())
        first = np.cumsum(ll) - ll
        pos = np.arange(tot, dtype=np.int64) + np.repeat(start[ii] - first, ll)
        out[o:o + tot] = flat[pos]
        o += tot
    thr = 1.0 / (12 * mean)
    for a in range(0, out.size, 1 << 26):
        seg = out[a:a + (1 << 26)]
        nl = rng.random(seg.size) < thr
        seg[(seg == 32) & nl] = 10
    while out.size < nbytes:
        out = np.concatenate([out, text_proxy(nbytes - out.size, seed + 1)])
    return out[:nbytes]


def _int_table(n: int, rng) -> np.ndarray:
    width = 4 if rng.random() < 0.5 else 8
    k = (n + width - 1) // width
    base = np.uint64(rng.integers(0, 1 << 20))
    vals = base + np.cumsum(rng.integers(0, 64, size=k)).astype(np.uint64)
    vals = (vals & np.uint64(0xFFFFFFFF)).astype("<u4") if width == 4 else vals.astype("<u8")
    return np.frombuffer(vals.tobytes(), dtype=np.uint8)[:n]


def _runs(n: int, rng) -> np.ndarray:
    out = np.empty(n, dtype=np.uint8)
    pos = 0
    while pos < n:
        ln = int(rng.integers(8, 2048))
        out[pos:pos + ln] = 0 if rng.random() < 0.6 else rng.integers(0, 256)
        pos += ln
    return out


def _records(n: int, rng) -> np.ndarray:
    # fixed-size records: small header + counters + a few random bytes
    rec = 32
    k = (n + rec - 1) // rec
    arr = np.zeros((k, rec), dtype=np.uint8)
    arr[:, 0:4] = np.frombuffer(b"REC\x01", dtype=np.uint8)
    ids = np.arange(k, dtype="<u4")
    arr[:, 4:8] = ids.view(np.uint8).reshape(k, 4)
    arr[:, 8:16] = rng.integers(0, 4, size=(k, 8), dtype=np.uint8)
    arr[:, 16:20] = rng.integers(0, 256, size=(k, 4), dtype=np.uint8)
    return arr.reshape(-1)[:n]


def silesia_proxy(nbytes: int, seed: int = 0x5157, chunk: int = 65536) -> np.ndarray:
    """Mixed-class corpus: each `chunk` bytes is one class (LZ4 ratio ~2)."""
    rng = np.random.default_rng(seed)
    jpg = np.frombuffer(_jpeg(), dtype=np.uint8)
    nchunks = (nbytes + chunk - 1) // chunk
    text = text_proxy(nchunks * chunk, seed ^ 0x1111)
    out = np.empty(nchunks * chunk, dtype=np.uint8)
    classes = rng.choice(6, size=nchunks, p=[0.40, 0.15, 0.10, 0.10, 0.10, 0.15])
    for i, c in enumerate(classes):
        lo, hi = i * chunk, (i + 1) * chunk
        if c == 0:
            out[lo:hi] = text[lo:hi]
        elif c == 1:
            out[lo:hi] = _int_table(chunk, rng)
        elif c == 2:
            out[lo:hi] = _runs(chunk, rng)
        elif c == 3:
            out[lo:hi] = rng.integers(0, 256, size=chunk, dtype=np.uint8)
        elif c == 4:
            s = int(rng.integers(0, max(1, jpg.size - chunk)))
            piece = jpg[s:s + chunk]
            out[lo:lo + piece.size] = piece
            if piece.size < chunk:
                out[lo + piece.size:hi] = 0
        else:
            out[lo:hi] = _records(chunk, rng)
    return out[:nbytes]


def fio_pattern(nbytes: int, seed: int = 0xF10) -> np.ndarray:
    """fio buffer_compress_percentage=50, buffer_compress_chunk=512."""
    rng = np.random.default_rng(seed)
    k = (nbytes + 511) // 512
    arr = np.zeros((k, 512), dtype=np.uint8)
    arr[:, :256] = rng.integers(0, 256, size=(k, 256), dtype=np.uint8)
    return arr.reshape(-1)[:nbytes]
