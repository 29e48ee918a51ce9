"""CPU tests of the oracle (the CPU restatement of the reference path).

The oracle is pinned against the reference's own outputs recorded in
SURVEY.md section 8c (tests/golden/reference_kat.json): nine frame
known-answers (size + SHA-256) over the reference's test_files with the
scatter-gather layouts the reference saw, and the decompressor's return
codes.  The remaining tests check properties the reference guarantees
(layout-class invariance, SG == linear, round trips, edge cases of
lz4e/lz4e_compress.c and lz4e/lz4e_decompress.c).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_ref
from lz4e_amd import BYU16, BYU32, compress_bound, corpus, make_sg

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KAT = json.load(open(os.path.join(GOLDEN, "reference_kat.json")))


def _kat_input(case, files):
    return files[case["file"]][case["start"]:case["start"] + case["len"]]


@pytest.mark.parametrize("case", KAT["compress"], ids=lambda c: f'{c["file"]}-{len(c["segments"])}x')
def test_reference_frames_linear(case, test_files):
    data = _kat_input(case, test_files)
    r, frame, _, _ = oracle_ref.compress(data, case["table_type"])
    assert r == case["size"]
    assert hashlib.sha256(frame).hexdigest() == case["sha256"]


@pytest.mark.parametrize("case", KAT["compress"], ids=lambda c: f'{c["file"]}-{len(c["segments"])}x')
def test_reference_frames_sg(case, test_files):
    """Same frames through the bio_vec API with the reference's SG layouts."""
    data = _kat_input(case, test_files)
    src = make_sg(data, case["segments"], shuffle_seed=len(case["segments"]))
    assert oracle_ref.table_type(src) == case["table_type"]
    cap = compress_bound(len(data))
    npages = -(-cap // 4096)
    dst = make_sg(b"", [4096] * npages, capacity=cap)
    r = oracle_ref.compress_sg(src, dst)
    assert r == case["size"]
    frame = dst.read_prefix(r)
    assert hashlib.sha256(frame).hexdigest() == case["sha256"]


def test_reference_decompress_codes(test_files):
    d = KAT["decompress"]
    data = test_files[d["frame"]["file"]][:d["frame"]["len"]]
    r, frame, _, _ = oracle_ref.compress(data, d["frame"]["table_type"])
    assert r == d["frame"]["size"]
    for c in d["cases"]:
        ret, out = oracle_ref.decompress(frame[:c["csize"]], c["cap"], csize=c["csize"])
        assert ret == c["ret"], c["what"]
        if ret > 0:
            assert out == data
    for c in d["single_zero_byte"]:
        assert oracle_ref.decompress(b"\x00", c["cap"])[0] == c["ret"]


def test_edge_empty_and_tiny():
    r, frame, fs, lr = oracle_ref.compress(b"", BYU16)
    assert (r, frame) == (1, b"\x00")
    for n in range(1, 13):
        data = bytes(range(100, 100 + n))
        r, frame, fs, lr = oracle_ref.compress(data, BYU16)
        assert frame == bytes([n << 4]) + data  # literals only (lz4e_compress.c:268-271)
        assert fs == 0 and lr == n
    # n == 13 is the first size that runs the match finder
    r, frame, _, _ = oracle_ref.compress(b"a" * 13, BYU16)
    assert oracle_ref.decompress(frame, 13) == (13, b"a" * 13)


def test_edge_limited_output(test_files):
    data = test_files["01.txt"][:4096]
    full = oracle_ref.compress(data, BYU16)
    assert full[0] == 2411
    # capacity below the bound but above the frame: same bytes (limitedOutput)
    assert oracle_ref.compress(data, BYU16, cap=2500)[:2] == full[:2]
    assert oracle_ref.compress(data, BYU16, cap=2411)[:2] == full[:2]
    assert oracle_ref.compress(data, BYU16, cap=2000)[0] == 0
    assert oracle_ref.compress(b"", BYU16, cap=0)[0] == 0


def test_edge_segment_limit():
    data = bytes(np.random.default_rng(1).integers(0, 4, 256 * 16, dtype=np.uint8))
    dst_cap = compress_bound(len(data))
    ok = make_sg(data, [16] * 256)
    assert oracle_ref.table_type(ok) == BYU32
    assert oracle_ref.compress_sg(ok, make_sg(b"", [dst_cap], capacity=dst_cap)) > 0
    data2 = data + b"x" * 16
    bad = make_sg(data2, [16] * 257)
    assert oracle_ref.table_type(bad) == 0
    assert oracle_ref.compress_sg(bad, make_sg(b"", [dst_cap + 64], capacity=dst_cap + 64)) == 0


def _random_layout(rng, n, cls):
    """Segment lengths giving table class `cls` for n bytes."""
    segs = []
    left = n
    if cls == BYU16:
        k = int(rng.integers(max(1, -(-n // 4096)), 17))
        cuts = np.sort(rng.choice(np.arange(1, n), size=k - 1, replace=False)) if k > 1 else []
        edges = [0, *cuts, n]
        segs = [int(b - a) for a, b in zip(edges[:-1], edges[1:])]
        if max(segs) > 4096:
            segs = [4096] * (n // 4096) + ([n % 4096] if n % 4096 else [])
        return segs
    while left:
        s = int(rng.integers(1, 8192))
        s = min(s, left)
        segs.append(s)
        left -= s
    if len(segs) < 17 and max(segs) <= 4096:
        segs = [1] * 16 + [n - 16]
    return segs


@pytest.mark.parametrize("seed", range(6))
def test_sg_equals_linear_and_layout_invariance(seed, test_files):
    rng = np.random.default_rng(seed)
    base = test_files["02.txt"] + test_files["03.jpg"][:20000]
    n = int(rng.integers(4000, 36000))
    start = int(rng.integers(0, len(base) - n))
    data = base[start:start + n]
    for cls in (BYU16, BYU32):
        expect = oracle_ref.compress(data, cls)
        for trial in range(3):
            segs = _random_layout(rng, n, cls)
            offs = [int(rng.integers(0, 4096)) for _ in segs]
            src = make_sg(data, segs, offsets=offs, shuffle_seed=trial)
            assert oracle_ref.table_type(src) == cls
            cap = compress_bound(n)
            dst = make_sg(b"", [512] * (-(-cap // 512)), capacity=cap, shuffle_seed=trial + 7)
            r = oracle_ref.compress_sg(src, dst)
            assert r == expect[0]
            assert dst.read_prefix(r) == expect[1]
            # iterator post-state (lz4e_compress.c:528 passes dstIter by value)
            assert src.it.bi_size == n - expect[2]
            assert dst.it.bi_size == cap - (r - expect[3])


def test_mid_segment_start():
    """Start iterator inside the first bvec (bi_bvec_done != 0)."""
    rng = np.random.default_rng(5)
    data = bytes(rng.integers(0, 3, 9000, dtype=np.uint8))
    src = make_sg(data, [4096, 4096, 4096], start_done=1000)
    assert src.read() == data
    assert oracle_ref.table_type(src) == BYU16
    cap = compress_bound(len(data))
    dst = make_sg(b"", [cap], capacity=cap)
    r = oracle_ref.compress_sg(src, dst)
    assert (r, dst.read_prefix(r)) == oracle_ref.compress(data, BYU16)[:2]


@pytest.mark.parametrize("kind", ["text", "runs", "random", "ints", "mixed"])
def test_oracle_roundtrip(kind):
    from lz4e_amd import corpus
    rng = np.random.default_rng(11)
    n = 70000
    if kind == "text":
        data = corpus.text_proxy(n, 3).tobytes()
    elif kind == "runs":
        data = corpus._runs(n, rng).tobytes()
    elif kind == "random":
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    elif kind == "ints":
        data = corpus._int_table(n, rng).tobytes()
    else:
        data = corpus.silesia_proxy(n, 9).tobytes()
    for cls, m in ((BYU16, 65536), (BYU32, n)):
        blk = data[:m]
        r, frame, _, _ = oracle_ref.compress(blk, cls)
        assert 0 < r <= compress_bound(m)
        assert oracle_ref.decompress(frame, m) == (m, blk)


def test_decompress_rejects_corruption():
    rng = np.random.default_rng(2)
    from lz4e_amd import corpus
    data = corpus.text_proxy(20000, 4).tobytes()
    r, frame, _, _ = oracle_ref.compress(data, BYU16)
    # truncations always fail; the error position never exceeds the input
    for cut in rng.integers(1, r, 40):
        ret, _ = oracle_ref.decompress(frame[:cut], len(data))
        assert ret < 0 and -ret - 1 <= cut
    # offset 0 decodes to zeros (LZ4_write32(op, offset), lz4e_decompress.c:313)
    assert oracle_ref.decompress(bytes([0x00, 0x00, 0x00, 0x50]) + b"abcde", 100) == (9, b"\0" * 4 + b"abcde")
    # an offset reaching before the block start fails at ip = 3 (:299-302)
    assert oracle_ref.decompress(bytes([0x00, 0x01, 0x00, 0x50]) + b"abcde", 100)[0] == -4


def test_sg_batch_equals_linear_batch():
    """The CPU baseline's two variants (bench.py cpu_baseline / _sg) compute
    the same frames: the faithful SG walk over 4 KiB and 512 B segments."""
    L = oracle_ref.load()
    nb, bs = 12, 65536
    data = corpus.silesia_proxy(nb * bs, 9)
    offs = np.arange(nb, dtype=np.uint64) * bs
    lens = np.full(nb, bs, np.uint32)
    cap = bs + bs // 255 + 16
    caps = np.full(nb, cap, np.uint32)
    slot = (cap + 64 + 15) // 16 * 16
    doffs = np.arange(nb, dtype=np.uint64) * slot
    for seg, tt in ((4096, 1), (512, 3)):
        o1, r1 = np.zeros(nb * slot, np.uint8), np.zeros(nb, np.int32)
        o2, r2 = np.zeros(nb * slot, np.uint8), np.zeros(nb, np.int32)
        tts = np.full(nb, tt, np.uint8)
        L.oracle_compress_linear_batch(data.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                       tts.ctypes.data, o1.ctypes.data,
                                       doffs.ctypes.data, caps.ctypes.data, r1.ctypes.data, nb, 4)
        L.oracle_compress_sg_batch(data.ctypes.data, offs.ctypes.data, lens.ctypes.data, seg,
                                   o2.ctypes.data, doffs.ctypes.data, caps.ctypes.data, r2.ctypes.data,
                                   nb, 4)
        assert (r1 == r2).all() and (r1 > 0).all()
        assert np.array_equal(o1, o2)


# ---------------------------------------------------------------------------
# dictionary mode (LZ4E extension of the reference's
# stubbed dict path -- no reference run pins these frames: parity unpinned)
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("n", [0, 12, 13, 4096, 65536])
@pytest.mark.parametrize("dsize", [0, 7, 8, 1000, 65536, 90000])
def test_dict_round_trip(n, dsize):
    data = corpus.silesia_proxy(n + dsize + 65536, 31).tobytes()
    dic, blk = data[:dsize], data[dsize:dsize + n]
    r, f = oracle_ref.compress_dict(blk, dic)
    assert r > 0
    assert oracle_ref.decompress_dict(f, n, dic) == (n, blk)
    # the decoder reads at most the last 64 KiB of the dictionary
    assert oracle_ref.decompress_dict(f, n, dic[-65536:]) == (n, blk)
    if dsize < 8:
        # under 8 bytes the dictionary is ignored (LZ4_loadDict): byU32 noDict frame
        assert f == oracle_ref.compress(blk, BYU32)[1]


def test_dict_helps_and_is_needed():
    data = corpus.text_proxy(3 * 65536, 5).tobytes()
    dic, blk = data[:65536], data[65536:131072]
    r0 = oracle_ref.compress(blk, BYU32)[0]
    r, f = oracle_ref.compress_dict(blk, dic)
    assert r < r0  # the dictionary's history shortens the frame
    # without (or with too short) a dictionary the frame references before
    # the output: the offset check of lz4e_decompress.c:299-302 fails it
    assert oracle_ref.decompress(f, len(blk))[0] < 0
    assert oracle_ref.decompress_dict(f, len(blk), dic[-16:])[0] < 0


def test_dict_decoder_offset_check():
    """extDict semantics: a match may reach dictSize bytes before the output;
    one byte further fails at the offset's position (checkOffset, :93, :299)
    unless the dictionary is 64 KiB or more (no check)."""
    frame = bytes([0x00, 0x05, 0x00, 0x50]) + b"abcde"  # match of 4 at offset 5, then 5 literals
    assert oracle_ref.decompress_dict(frame, 100, b"XYZUV") == (9, b"XYZU" + b"abcde")
    assert oracle_ref.decompress_dict(frame, 100, b"YZUV")[0] == -4
    big = bytes(range(256)) * 256  # 64 KiB
    assert oracle_ref.decompress_dict(frame, 100, big)[0] == 9
