"""GPU parity tests: the HIP path, called through the C ABI, against the CPU
oracle on the same seeded inputs.  Integer/byte work, so the bar is
bit-exact: identical return values, identical frame bytes, identical
iterator post-state, identical decoder error codes."""
import ctypes
import hashlib
import zlib
import json
import os

import numpy as np
import pytest

import oracle_ref
from lz4e_amd import BYU16, BYU32, BYU64, compress_bound, corpus, make_sg

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KAT = json.load(open(os.path.join(GOLDEN, "reference_kat.json")))


def _corpus(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "text":
        return corpus.text_proxy(n, seed)
    if kind == "runs":
        return corpus._runs(n, rng)
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8)
    if kind == "ints":
        return corpus._int_table(n, rng)
    if kind == "fio":
        return corpus.fio_pattern(n, seed)
    if kind == "small_alpha":
        return rng.integers(0, 3, n, dtype=np.uint8)
    return corpus.silesia_proxy(n, seed)


# ---------------------------------------------------------------------------
# device batch helpers
# ---------------------------------------------------------------------------

def _gpu_compress(amd, blocks, ttypes, caps=None):
    import torch
    n = len(blocks)
    lens = np.array([len(b) for b in blocks], dtype=np.int64)
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum((lens + 15) // 16 * 16)[:-1]
    total = int(offs[-1] + lens[-1]) + 16 if n else 16
    host = np.zeros(total, dtype=np.uint8)
    for i, b in enumerate(blocks):
        host[offs[i]:offs[i] + lens[i]] = np.frombuffer(bytes(b), dtype=np.uint8)
    bounds = lens + lens // 255 + 16
    caps = bounds if caps is None else np.asarray(caps, dtype=np.int64)
    slot = np.minimum(caps, bounds) + 64
    doffs = np.zeros(n, dtype=np.int64)
    doffs[1:] = np.cumsum((slot + 15) // 16 * 16)[:-1]
    dev = torch.device("cuda")
    src = torch.from_numpy(host).to(dev)
    dst = torch.zeros(int(doffs[-1] + slot[-1]) + 16, dtype=torch.uint8, device=dev)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).to(dev)
    ret = torch.full((n,), -7, dtype=torch.int32, device=dev)
    aux = torch.zeros(2 * n, dtype=torch.int32, device=dev)
    amd.compress_batch_dev(src, t(offs, np.int64), t(lens, np.int32), t(ttypes, np.uint8), dst,
                           t(doffs, np.int64), t(caps, np.int32), ret, aux)
    torch.cuda.synchronize()
    r = ret.cpu().numpy()
    d = dst.cpu().numpy()
    ax = aux.cpu().numpy().reshape(-1, 2)
    frames = [d[doffs[i]:doffs[i] + max(r[i], 0)].tobytes() for i in range(n)]
    return r, frames, ax


DEC_AUTO, DEC_WAVE, DEC_PIPE, DEC_SMALL, DEC_GROUP = 0, 1, 2, 6, 7
DEC_GROUP_NB = 9  # the group decoder without its hand-over (every block decoded by its group)


def _gpu_decompress(amd, frames, caps, csizes=None, max_cap=None, mode=DEC_AUTO):
    """Decode on the GPU; mode forces a decoder (one wave per block, or the
    pipelined 4-wave one) through the diagnostic entry point."""
    import torch
    n = len(frames)
    csizes = [len(f) for f in frames] if csizes is None else csizes
    flen = np.array([len(f) for f in frames], dtype=np.int64)
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum((flen + 15) // 16 * 16 + 16)[:-1]
    host = np.zeros(int(offs[-1] + flen[-1]) + 16 if n else 16, dtype=np.uint8)
    for i, f in enumerate(frames):
        host[offs[i]:offs[i] + flen[i]] = np.frombuffer(bytes(f), dtype=np.uint8)
    caps = np.asarray(caps, dtype=np.int64)
    slot = np.maximum(caps, 0) + 64
    doffs = np.zeros(n, dtype=np.int64)
    doffs[1:] = np.cumsum((slot + 15) // 16 * 16)[:-1]
    dev = torch.device("cuda")
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).to(dev)
    src = torch.from_numpy(host).to(dev)
    dst = torch.zeros(int(doffs[-1] + slot[-1]) + 16, dtype=torch.uint8, device=dev)
    ret = torch.full((n,), -7777, dtype=torch.int32, device=dev)
    if mode == DEC_AUTO:
        amd.decompress_batch_dev(src, t(offs, np.int64), t(csizes, np.int32), dst, t(doffs, np.int64),
                                 t(caps, np.int32), ret, max_cap=max_cap)
    else:
        L = amd.lib()
        P = ctypes.c_void_p
        L.lz4e_debug_decompress_stamped.argtypes = [P] * 7 + [ctypes.c_uint32, P, P, ctypes.c_uint32,
                                                               ctypes.c_uint32]
        a = [t(offs, np.int64), t(csizes, np.int32), t(doffs, np.int64), t(caps, np.int32)]
        assert L.lz4e_debug_decompress_stamped(src.data_ptr(), a[0].data_ptr(), a[1].data_ptr(),
                                               dst.data_ptr(), a[2].data_ptr(), a[3].data_ptr(),
                                               ret.data_ptr(), n, None, None, 0, mode) == 0
    torch.cuda.synchronize()
    r = ret.cpu().numpy()
    d = dst.cpu().numpy()
    return r, [d[doffs[i]:doffs[i] + max(r[i], 0)].tobytes() for i in range(n)]


# ---------------------------------------------------------------------------
# reference known answers through the drop-in entry points
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("case", KAT["compress"], ids=lambda c: f'{c["file"]}-{len(c["segments"])}x')
def test_kat_frames_via_compress_default(gpu, case, test_files):
    data = test_files[case["file"]][case["start"]:case["start"] + case["len"]]
    cap = compress_bound(len(data))
    src = make_sg(data, case["segments"], shuffle_seed=1)
    dst = make_sg(b"", [4096] * (-(-cap // 4096)), capacity=cap, shuffle_seed=2)
    r = gpu.compress_default(src, dst)
    assert r == case["size"], gpu.last_error()
    assert hashlib.sha256(dst.read_prefix(r)).hexdigest() == case["sha256"]
    # iterator post-state identical to the oracle's
    src2 = make_sg(data, case["segments"], shuffle_seed=1)
    dst2 = make_sg(b"", [4096] * (-(-cap // 4096)), capacity=cap, shuffle_seed=2)
    assert oracle_ref.compress_sg(src2, dst2) == r
    assert src.it.as_tuple() == src2.it.as_tuple()
    assert dst.it.as_tuple() == dst2.it.as_tuple()


def test_kat_decompress_codes(gpu, test_files):
    d = KAT["decompress"]
    data = test_files[d["frame"]["file"]][:d["frame"]["len"]]
    frame = oracle_ref.compress(data, d["frame"]["table_type"])[1]
    for c in d["cases"]:
        ret, out = gpu.decompress_safe(frame[:c["csize"]], c["cap"], compressed_size=c["csize"])
        assert ret == c["ret"], c["what"]
        if ret > 0:
            assert out == data
    for c in d["single_zero_byte"]:
        assert gpu.decompress_safe(b"\x00", c["cap"])[0] == c["ret"]


def test_edge_cases_compress_default(gpu):
    for n in list(range(0, 20)) + [255, 256, 4095, 4096, 4097]:
        data = _corpus("small_alpha", n, n).tobytes()
        src = make_sg(data, [n] if n else [1], capacity=n)
        cap = compress_bound(n)
        dst = make_sg(b"", [cap + 8], capacity=cap)
        cls = oracle_ref.table_type(src) if n >= 13 else BYU16
        r = gpu.compress_default(src, dst)
        assert (r, dst.read_prefix(r)) == oracle_ref.compress(data, cls)[:2], n
    # 256 segments OK, 257 -> 0 (lz4e_compress.c:197-198, :274-277)
    data = _corpus("small_alpha", 16 * 257, 3).tobytes()
    cap = compress_bound(len(data))
    ok = make_sg(data[:16 * 256], [16] * 256)
    r = gpu.compress_default(ok, make_sg(b"", [cap], capacity=cap))
    assert r == oracle_ref.compress(data[:16 * 256], BYU32)[0]
    bad = make_sg(data, [16] * 257)
    assert gpu.compress_default(bad, make_sg(b"", [cap], capacity=cap)) == 0
    assert bad.it.bi_size == len(data)


# ---------------------------------------------------------------------------
# randomized batches against the oracle
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("kind", ["mixed", "text", "runs", "random", "ints", "fio", "small_alpha"])
@pytest.mark.parametrize("cls", [BYU16, BYU32])
def test_compress_batch_vs_oracle(gpu, kind, cls):
    rng = np.random.default_rng(zlib.crc32(f"{kind}-{cls}".encode()))
    data = _corpus(kind, 1 << 21, 17)
    lens = [int(x) for x in rng.choice([0, 1, 12, 13, 14, 100, 4096, 4097, 30000, 65535, 65536], size=48)]
    if cls == BYU32:
        lens += [65537, 131072, 200000]
    blocks, starts = [], []
    for ln in lens:
        s = int(rng.integers(0, data.size - ln))
        blocks.append(data[s:s + ln].tobytes())
    ttypes = [cls] * len(blocks)
    r, frames, aux = _gpu_compress(gpu, blocks, ttypes)
    for i, b in enumerate(blocks):
        er, ef, efs, elr = oracle_ref.compress(b, cls)
        assert r[i] == er, (i, len(b))
        assert frames[i] == ef, (i, len(b))
        assert (aux[i][0], aux[i][1]) == (efs, elr), (i, len(b))


@pytest.mark.parametrize("cls", [BYU16, BYU32])
def test_compress_search_handover_patterns(gpu, cls):
    """Blocks of [R random bytes | Z equal bytes] chunks: after each match the
    rematch misses and the search runs through its window, hands over to the
    generic skip-step search at probe 48 and finds the next run at a probe
    number set by R -- before, at and after the hand-over, with the block end
    (mflimit) landing inside the search for the truncated lengths.  LDS-staged
    (<= 4 KiB) and HBM blocks; frames, sizes and iterator post-state equal the
    oracle's."""
    rng = np.random.default_rng(4801 + cls)
    blocks = []
    for R in (20, 40, 47, 48, 49, 55, 60, 64, 66, 70, 100, 130, 200, 300):
        for Z in (13, 64, 256):
            unit = np.concatenate([rng.integers(0, 256, R, dtype=np.uint8), np.full(Z, 7, np.uint8)])
            data = np.tile(unit, 65536 // unit.size + 2)
            for ln in (4096, 4095, 3000, 2500, 20000, 65536):
                if cls == BYU16 or ln != 4095:
                    blocks.append(data[:ln].tobytes())
    r, frames, aux = _gpu_compress(gpu, blocks, [cls] * len(blocks))
    for i, b in enumerate(blocks):
        er, ef, efs, elr = oracle_ref.compress(b, cls)
        assert r[i] == er, (i, len(b))
        assert frames[i] == ef, (i, len(b))
        assert (aux[i][0], aux[i][1]) == (efs, elr), (i, len(b))


def test_compress_byu64(gpu):
    """byU64 class (a > 16 MiB segment): HBM-resident path, 2048-entry table."""
    n = (1 << 24) + 40000
    data = _corpus("mixed", n, 5).tobytes()
    r, frames, _ = _gpu_compress(gpu, [data], [BYU64])
    er, ef, _, _ = oracle_ref.compress(data, BYU64)
    assert r[0] == er
    assert frames[0] == ef


@pytest.mark.parametrize("kind", ["text", "mixed", "random"])
def test_compress_limited_output(gpu, kind):
    """Capacities below LZ4E_COMPRESSBOUND take the limitedOutput checks."""
    data = _corpus(kind, 1 << 20, 23)
    rng = np.random.default_rng(7)
    blocks, caps, ttypes = [], [], []
    for i in range(40):
        ln = int(rng.choice([4096, 20000, 65536]))
        s = int(rng.integers(0, data.size - ln))
        b = data[s:s + ln].tobytes()
        full = oracle_ref.compress(b, BYU16)[0]
        cap = int(max(0, full + rng.integers(-40, 12)))
        blocks.append(b)
        caps.append(min(cap, compress_bound(ln)))
        ttypes.append(BYU16)
    r, frames, _ = _gpu_compress(gpu, blocks, ttypes, caps)
    for i, b in enumerate(blocks):
        er, ef, _, _ = oracle_ref.compress(b, BYU16, cap=caps[i])
        assert r[i] == er, (i, caps[i])
        assert frames[i] == ef


def test_compress_sg_batch_layouts(gpu):
    rng = np.random.default_rng(99)
    data = _corpus("mixed", 1 << 20, 31).tobytes()
    pairs, twins = [], []
    for i in range(24):
        n = int(rng.integers(13, 60000))
        s = int(rng.integers(0, len(data) - n))
        blk = data[s:s + n]
        if i % 2:
            segs = [min(4096, n - k) for k in range(0, n, 4096)]
        else:
            segs = [min(512, n - k) for k in range(0, n, 512)]
        offs = [int(rng.integers(0, 4096)) for _ in segs]
        cap = compress_bound(n)
        mk = lambda seed: (make_sg(blk, segs, offsets=offs, shuffle_seed=seed),
                           make_sg(b"", [1000] * (-(-cap // 1000)), capacity=cap, shuffle_seed=seed))
        pairs.append(mk(i))
        twins.append(mk(i))
    rets = gpu.compress_sg_batch(pairs)
    for (s, d), (s2, d2), r in zip(pairs, twins, rets):
        er = oracle_ref.compress_sg(s2, d2)
        assert r == er
        assert d.read_prefix(r) == d2.read_prefix(er)
        assert s.it.as_tuple() == s2.it.as_tuple()
        assert d.it.as_tuple() == d2.it.as_tuple()


# ---------------------------------------------------------------------------
# decoder parity (values and error codes)
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("kind", ["mixed", "text", "runs", "random", "fio", "small_alpha"])
def test_decompress_batch_vs_oracle(gpu, kind):
    rng = np.random.default_rng(len(kind))
    data = _corpus(kind, 1 << 21, 41)
    frames, caps, expect = [], [], []
    for i in range(40):
        ln = int(rng.choice([1, 13, 100, 4096, 65536, 200000]))
        s = int(rng.integers(0, data.size - ln))
        b = data[s:s + ln].tobytes()
        f = oracle_ref.compress(b, BYU32 if ln > 65536 else BYU16)[1]
        frames.append(f)
        caps.append(ln + int(rng.choice([0, 0, 1, 100])))
        expect.append(b)
    r, outs = _gpu_decompress(gpu, frames, caps)
    for i in range(len(frames)):
        er, eo = oracle_ref.decompress(frames[i], caps[i])
        assert r[i] == er == len(expect[i])
        assert outs[i] == eo == expect[i]


@pytest.mark.parametrize("dec", [DEC_AUTO, DEC_PIPE, DEC_WAVE, DEC_SMALL, DEC_GROUP, DEC_GROUP_NB],
                         ids=["auto", "pipe", "wave", "small", "group", "group_nobail"])
@pytest.mark.parametrize("mode", ["truncate", "flip", "garbage", "small_cap", "csize"])
def test_decompress_error_codes(gpu, mode, dec):
    rng = np.random.default_rng(1234 + len(mode))
    data = _corpus("mixed", 1 << 20, 77)
    frames, caps, csizes = [], [], []
    for i in range(160):
        ln = int(rng.choice([50, 4096, 30000, 65536]))
        s = int(rng.integers(0, data.size - ln))
        f = bytearray(oracle_ref.compress(data[s:s + ln].tobytes(), BYU16)[1])
        cap, cs = ln, len(f)
        if mode == "truncate":
            cs = int(rng.integers(0, len(f)))
        elif mode == "flip":
            for _ in range(int(rng.integers(1, 4))):
                j = int(rng.integers(0, len(f)))
                f[j] ^= 1 << int(rng.integers(0, 8))
        elif mode == "garbage":
            f = bytearray(rng.integers(0, 256, int(rng.integers(1, 3000)), dtype=np.uint8).tobytes())
            cs = len(f)
        elif mode == "small_cap":
            cap = int(rng.integers(0, ln))
        else:
            cs = len(f) + int(rng.integers(-3, 0))
        frames.append(bytes(f))
        caps.append(cap)
        csizes.append(cs)
    r, outs = _gpu_decompress(gpu, frames, caps, csizes, mode=dec)
    for i in range(len(frames)):
        er, eo = oracle_ref.decompress(frames[i], caps[i], csize=csizes[i])
        assert r[i] == er, (i, mode, caps[i], csizes[i])
        if er >= 0:
            assert outs[i] == eo


def test_decompress_single_calls(gpu, test_files):
    for name in ("01.txt", "02.txt", "03.jpg"):
        data = test_files[name][:65536]
        f = oracle_ref.compress(data, BYU16)[1]
        assert gpu.decompress_safe(f, len(data)) == (len(data), data)
        res = gpu.decompress_batch([f, f[:-1], b""], [len(data), len(data), 10])
        assert res[0] == (len(data), data)
        assert res[1][0] == oracle_ref.decompress(f[:-1], len(data))[0]
        assert res[2][0] == -1


@pytest.mark.parametrize("kind", ["fio", "mixed", "random", "head"])
def test_decompress_small_blocks_in_lds(gpu, kind):
    """Blocks of <= 4608 bytes: the one-wave decoder's LDS form (whole
    output in LDS) and the lane-per-block decoder with its hand-over to the
    one-wave decoder ("head": 230 random bytes and 200 zeros, then short
    sequences),
    and auto mode: exact and +32 capacities, truncations and short
    capacities, values and bytes equal the oracle's."""
    rng = np.random.default_rng(4608 + len(kind))
    data = _corpus("mixed" if kind == "head" else kind, 1 << 21, 91)
    rnd = rng.integers(0, 256, 230, dtype=np.uint8).tobytes() + bytes(200)
    frames, caps, want = [], [], []
    for i in range(3000):
        n = int(rng.choice([4096, 4096, int(rng.integers(1, 4609))]))
        s0 = int(rng.integers(0, data.size - n))
        blk = data[s0:s0 + n].tobytes()
        if kind == "head":  # a long first sequence, then short ones (lane hand-over mid-block)
            blk = (rnd + blk)[:n]
        f = oracle_ref.compress(blk, BYU16)[1]
        cap = n + (32 if i % 4 == 1 else 0)
        if i % 9 == 2:
            f = f[:int(rng.integers(1, len(f)))]
        elif i % 9 == 5:
            cap = max(0, n - int(rng.integers(1, 40)))
        frames.append(f)
        caps.append(cap)
        want.append(oracle_ref.decompress(f, cap))
    for mode in (DEC_AUTO, DEC_SMALL, DEC_GROUP):
        r, outs = _gpu_decompress(gpu, frames, caps, max_cap=max(caps), mode=mode)
        for i, (er, eb) in enumerate(want):
            assert r[i] == er, (mode, i, r[i], er)
            if er >= 0:
                assert outs[i] == eb, (mode, i)


# ---------------------------------------------------------------------------
# full-size property: GPU round trip of the benchmark workload shape
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("cls,bs,kind", [(BYU16, 65536, "mixed"), (BYU16, 4096, "fio"),
                                         (BYU32, 65536, "mixed"), (BYU32, 262144, "text")])
def test_full_size_roundtrip(gpu, cls, bs, kind):
    n_blocks = {65536: 256, 4096: 2048, 262144: 32}[bs]
    data = _corpus(kind, n_blocks * bs, 2024)
    blocks = [data[i * bs:(i + 1) * bs].tobytes() for i in range(n_blocks)]
    r, frames, _ = _gpu_compress(gpu, blocks, [cls] * n_blocks)
    assert (r > 0).all()
    dr, outs = _gpu_decompress(gpu, frames, [bs] * n_blocks)
    assert (dr == bs).all()
    assert all(o == b for o, b in zip(outs, blocks))
    # the oracle on every 8th block: identical frames
    for i in range(0, n_blocks, 8):
        assert frames[i] == oracle_ref.compress(blocks[i], cls)[1]


@pytest.mark.parametrize("mode", [DEC_WAVE, DEC_PIPE, DEC_GROUP_NB], ids=["wave", "pipe", "group_nobail"])
def test_decompress_huge_runs(gpu, mode):
    """Blocks whose sequences are hundreds of MiB long: a 256 MiB run of one
    byte (a single match whose length extension is ~1 MiB of 0xFF) and a
    96 MiB literal run followed by a 160 MiB run.  Both decoders copy them
    in HBM; on the pipelined one the other waves wait on that copy for
    ~0.1 s, which the watchdog must not mistake for a hang (its count resets
    on every heartbeat of the copy).  Frames from the oracle
    (lz4e_compress.c restated), values and bytes checked in full."""
    run = b"\xab" * (256 << 20)
    rnd = np.random.default_rng(8).integers(0, 256, 96 << 20, dtype=np.uint8).tobytes()
    blocks = [run, rnd + run[:160 << 20]]
    frames = [oracle_ref.compress(b, BYU32)[1] for b in blocks]
    r, outs = _gpu_decompress(gpu, frames, [len(b) for b in blocks], mode=mode)
    for i, b in enumerate(blocks):
        assert r[i] == len(b), (i, r[i])
        assert outs[i] == b, i


def test_pipe_decoder_watchdog_valid_worst_case(gpu):
    """The pipelined decoder's watchdog (decompress_pipe_kernel, DESIGN.md §3
    "Watchdog") on valid worst-case frames under a full-chip batch: 2 048
    blocks of 256 KiB -- runs of one byte (one offset-1 match with a ~1 KiB
    match-length extension), incompressible data (a ~1 KiB literal-length
    extension), text and records -- forced onto the pipelined decoder (6
    workgroups per CU, two rounds of them).  Every block returns the
    oracle's value (its size), never LZ4E_DECODE_ABORTED, and its bytes."""
    import torch
    bs, n = 262144, 2048
    rng = np.random.default_rng(5)
    srcs = [b"\x5a" * bs, rng.integers(0, 256, bs, dtype=np.uint8).tobytes(),
            _corpus("text", bs, 3).tobytes(), _corpus("mixed", bs, 4).tobytes()]
    frames = [oracle_ref.compress(b, BYU32)[1] for b in srcs]
    for b, f in zip(srcs, frames):
        assert oracle_ref.decompress(f, bs) == (bs, b)
    dev = torch.device("cuda")
    slot = (bs + bs // 255 + 16 + 15) // 16 * 16
    src = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    for i in range(4):
        src[i * slot:i * slot + len(frames[i])] = torch.frombuffer(bytearray(frames[i]), dtype=torch.uint8).to(dev)
    for i in range(4, n):  # (block i: copy of block i % 4)
        j = i % 4
        src[i * slot:i * slot + len(frames[j])] = src[j * slot:j * slot + len(frames[j])]
    soff = torch.arange(n, dtype=torch.int64, device=dev) * slot
    clen = torch.tensor([len(frames[i % 4]) for i in range(n)], dtype=torch.int32, device=dev)
    doff = torch.arange(n, dtype=torch.int64, device=dev) * bs
    caps = torch.full((n,), bs, dtype=torch.int32, device=dev)
    out = torch.zeros(n * bs + 64, dtype=torch.uint8, device=dev)
    ret = torch.full((n,), -7777, dtype=torch.int32, device=dev)
    L = gpu.lib()
    P = ctypes.c_void_p
    L.lz4e_debug_decompress_stamped.argtypes = [P] * 7 + [ctypes.c_uint32, P, P, ctypes.c_uint32, ctypes.c_uint32]
    assert L.lz4e_debug_decompress_stamped(src.data_ptr(), soff.data_ptr(), clen.data_ptr(), out.data_ptr(),
                                           doff.data_ptr(), caps.data_ptr(), ret.data_ptr(), n, None, None,
                                           bs, DEC_PIPE) == 0
    torch.cuda.synchronize()
    assert (ret == bs).all(), ret[ret != bs][:8].tolist()
    want = [torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev) for b in srcs]
    for i in range(n):
        assert torch.equal(out[i * bs:(i + 1) * bs], want[i % 4]), i


@pytest.mark.parametrize("mode", [DEC_WAVE, DEC_PIPE, DEC_GROUP_NB], ids=["wave", "pipe", "group_nobail"])
@pytest.mark.parametrize("cap_extra", [0, 100000])
def test_decompress_periodic_matches(gpu, cap_extra, mode):
    """Self-overlapping matches of every period 1..40 and lengths around
    1x-3x the period (the overlap-copy cases), on both decoders.  With the
    exact capacity the last sequences fall inside the reference's
    end-of-output margins (op > oend - 32 / oend - 12: no shortcut, exact end
    checks, lz4e_decompress.c:150-191, 223-288, 422-431) and take the scalar
    path; with 100 KB spare they stay on the fast path (span-staged)."""
    rng = np.random.default_rng(99)
    frames, caps, expect = [], [], []
    for period in range(1, 41):
        parts = []
        for rep in (1, 2, 3, 5, 9, 17, 40, 200):
            parts.append(rng.integers(0, 256, 37, dtype=np.uint8).tobytes())
            unit = rng.integers(0, 256, period, dtype=np.uint8).tobytes()
            parts.append((unit * (rep + 2))[:period * rep + int(rng.integers(0, period))])
        b = b"".join(parts) + rng.integers(0, 256, 20, dtype=np.uint8).tobytes()
        frames.append(oracle_ref.compress(b, BYU16)[1])
        caps.append(len(b) + cap_extra)
        expect.append(b)
    r, outs = _gpu_decompress(gpu, frames, caps, mode=mode)
    for i in range(len(frames)):
        assert r[i] == len(expect[i]), i
        assert outs[i] == expect[i], i


# ---------------------------------------------------------------------------
# chunk-layer write round trip (lz4e_bdev/lz4e_req.c:144-213)
# ---------------------------------------------------------------------------

def _chunk_check(gpu, srcs, payloads, want_frames=True):
    stats = gpu.ChunkStats()
    good, res = gpu.chunk_write_batch(srcs, want_frames=want_frames, stats=stats)
    nfail = 0
    for s, blk, (status, csize, data, frame) in zip(srcs, payloads, res):
        tt = gpu.table_type(s)
        if tt == 0:  # > BIO_MAX_VECS segments: LZ4E_compress_default returns 0 -> -EIO
            assert status == -gpu.EIO and csize == 0
            nfail += 1
            continue
        er, ef, _, _ = oracle_ref.compress(blk, tt)
        assert status == 0 and csize == er
        assert data == blk
        if want_frames:
            assert frame == ef
    assert good == len(srcs) - nfail
    # only completed round trips count (lz4e_end_io, lz4e_req.c:231-246); a
    # request failing in lz4e_write_req_init touches no counter (lz4e_dev.c:187-202)
    assert stats.reqs_total == len(srcs) - nfail and stats.reqs_failed == 0
    # one merged bio_vec per successful non-empty request (lz4e_stats.c:47)
    assert stats.vec_count == sum(1 for s, b in zip(srcs, payloads) if gpu.table_type(s) and len(b))
    assert stats.data_in_bytes == sum(len(b) for s, b in zip(srcs, payloads) if gpu.table_type(s))
    return stats


def test_chunk_write_batch_layouts(gpu):
    rng = np.random.default_rng(404)
    data = _corpus("mixed", 1 << 20, 41).tobytes()
    srcs, payloads = [], []
    sizes = [0, 1, 12, 13, 100, 4096, 4096, 8192, 65536, 65536, 30001, 131072]
    for i, n in enumerate(sizes):
        s = int(rng.integers(0, len(data) - n))
        blk = data[s:s + n]
        seg = [4096, 512, 1000][i % 3]
        done = int(rng.integers(0, 64)) if i % 4 == 3 else 0
        segs = [min(seg, n + done - k) for k in range(0, n + done, seg)] or [16]
        offs = [int(rng.integers(0, 4096)) for _ in segs]
        srcs.append(make_sg(blk, segs, offsets=offs, start_done=done, shuffle_seed=i))
        payloads.append(blk)
    # 257 segments: rejected like the reference (lz4e_compress.c:274-277)
    blk = data[:257 * 16]
    srcs.append(make_sg(blk, [16] * 257))
    payloads.append(blk)
    _chunk_check(gpu, srcs, payloads)


def test_chunk_write_batch_streamed(gpu):
    """144 MiB of input through the pipeline twice: in 16 MiB sub-batches
    (nine, so the four slots cycle: a slot's results are handed out before
    it takes the next sub-batch) and in the default call-sized ones (four,
    all in flight together)."""
    bs, nreq = 65536, 2200
    data = corpus.silesia_proxy(nreq * bs, 0x5157)
    srcs, payloads = [], []
    for i in range(nreq):
        blk = data[i * bs:(i + 1) * bs].tobytes()
        srcs.append(make_sg(blk, [4096] * 16))
        payloads.append(blk)
    L = gpu.lib()
    L.lz4e_debug_chunk_sub_bytes.argtypes = [ctypes.c_uint64]
    for sub in (16 << 20, 0):
        L.lz4e_debug_chunk_sub_bytes(sub)
        try:
            stats = gpu.ChunkStats()
            good, res = gpu.chunk_write_batch(srcs, want_frames=True, stats=stats)
        finally:
            L.lz4e_debug_chunk_sub_bytes(0)
        assert good == nreq and stats.reqs_failed == 0
        assert all(st == 0 and d == b for (st, _, d, _), b in zip(res, payloads))
        for i in range(0, nreq, 157):
            er, ef, _, _ = oracle_ref.compress(payloads[i], BYU16)
            assert res[i][1] == er and res[i][3] == ef
        assert stats.frame_bytes == sum(r[1] for r in res)


# ---------------------------------------------------------------------------
# SG-output decompress
# ---------------------------------------------------------------------------

def test_decompress_sg_layouts_and_codes(gpu):
    rng = np.random.default_rng(808)
    data = _corpus("mixed", 1 << 20, 51).tobytes()
    frames, dsts, blocks, exp = [], [], [], []
    for i in range(16):
        n = int(rng.integers(0, 70000))
        s = int(rng.integers(0, len(data) - n))
        blk = data[s:s + n]
        er, ef, _, _ = oracle_ref.compress(blk, BYU16 if n <= 65536 else BYU32)
        if i % 5 == 4:
            ef = ef[:len(ef) // 2]  # truncated: the decoder's error code, nothing written
        cap = n + int(rng.integers(0, 3)) * 100
        seg = [512, 4096, 1000, 333][i % 4]
        done = int(rng.integers(0, 100)) if i % 3 == 2 else 0
        segs = [seg] * (-(-(cap + done) // seg) or 1)
        offs = [int(rng.integers(0, 4096)) for _ in segs]
        dsts.append(make_sg(b"", segs, offsets=offs, start_done=done, capacity=cap,
                            shuffle_seed=i, fill=0xA5))
        frames.append(ef)
        blocks.append(blk)
        exp.append(oracle_ref.decompress(ef, cap))
    before = [(d.it.as_tuple(), d.read_prefix(sum(d.bvecs[k].bv_len for k in range(d.nseg)))) for d in dsts]
    rets = gpu.decompress_sg_batch(frames, dsts)
    for d, blk, (er, eb), r, (it0, raw0) in zip(dsts, blocks, exp, rets, before):
        assert r == er
        if r < 0:
            assert d.it.as_tuple() == it0
            assert d.read_prefix(len(raw0)) == raw0
            continue
        assert r == len(blk)
        assert gather_from(d, it0, r) == blk
        assert d.it.bi_size == it0[0] - r


def gather_from(d, it0, n):
    """n bytes of d's segments starting at the ORIGINAL iterator position it0."""
    size, idx, done = it0
    out = bytearray()
    while len(out) < n:
        b = d.bvecs[idx]
        take = min(b.bv_len - done, n - len(out))
        out += ctypes.string_at(b.bv_page + b.bv_offset + done, take)
        done = 0
        idx += 1
    return bytes(out)


def test_decompress_safe_sg_single(gpu, test_files):
    blk = test_files["02.txt"]
    er, ef, _, _ = oracle_ref.compress(blk, BYU16)
    d = make_sg(b"", [512] * (-(-len(blk) // 512)), capacity=len(blk), shuffle_seed=3)
    assert gpu.decompress_safe_sg(ef, d) == len(blk)
    assert d.read_prefix(len(blk)) == blk
    assert d.it.bi_size == 0
    d2 = make_sg(b"", [4096] * 5, capacity=len(blk) - 1)
    assert gpu.decompress_safe_sg(ef, d2) == oracle_ref.decompress(ef, len(blk) - 1)[0] < 0


def test_chunk_write_batch_fault_then_smaller_call(gpu):
    """A pipeline failure part way through (injected after the first
    sub-batch is in flight) returns -1 with every request -EIO and the
    caller's stats untouched; the next, smaller call is unaffected by what
    the failed one left in flight."""
    bs, nreq = 65536, 1100  # four 18 MiB sub-batches
    data = corpus.silesia_proxy(nreq * bs, 77)
    srcs = [make_sg(data[i * bs:(i + 1) * bs].tobytes(), [4096] * 16) for i in range(nreq)]
    L = gpu.lib()
    L.lz4e_debug_chunk_fault_after.argtypes = [ctypes.c_int]
    stats = gpu.ChunkStats()
    L.lz4e_debug_chunk_fault_after(1)
    try:
        with pytest.raises(gpu.GpuUnavailable, match="injected"):
            gpu.chunk_write_batch(srcs, want_frames=True, stats=stats)
    finally:
        L.lz4e_debug_chunk_fault_after(-1)
    assert (stats.reqs_total, stats.reqs_failed, stats.vec_count, stats.data_in_bytes) == (0, 0, 0, 0)
    small = srcs[:5]
    good, res = gpu.chunk_write_batch(small, want_frames=True, stats=stats)
    assert good == 5 and stats.reqs_total == 5 and stats.vec_count == 5
    for i, (st, csize, d, fr) in enumerate(res):
        blk = data[i * bs:(i + 1) * bs].tobytes()
        er, ef, _, _ = oracle_ref.compress(blk, BYU16)
        assert st == 0 and csize == er and d == blk and fr == ef


def test_single_calls_concurrent(gpu, test_files):
    """LZ4E_compress_default / LZ4E_decompress_safe from 16 threads at once
    (the reference is reentrant given distinct wrkmem and is called from
    every submitting CPU, lz4e_dev.c:174 -> lz4e_req.c:177): concurrent
    calls are coalesced into shared batch launches, and every result --
    frame, iterator post-state, decoded bytes, error code -- equals the
    oracle's for its own request."""
    import threading
    pool = _corpus("mixed", 1 << 20, 5).tobytes()
    errors = []

    def worker(t):
        rng = np.random.default_rng(500 + t)
        try:
            for k in range(25):
                n = int(rng.integers(0, 20000)) if k % 5 else 4096
                s0 = int(rng.integers(0, len(pool) - n))
                blk = pool[s0:s0 + n]
                seg = [4096, 512][(t + k) % 2]
                segs = [min(seg, n - j) for j in range(0, n, seg)] or [16]
                src = make_sg(blk, segs, shuffle_seed=k)
                cap = compress_bound(n)
                dst = make_sg(b"", [4096] * (-(-cap // 4096) or 1), capacity=cap)
                tt = gpu.table_type(src)
                er, ef, fs, lr = oracle_ref.compress(blk, tt if n >= 13 else BYU16)
                r = gpu.compress_default(src, dst)
                if r != er or dst.read_prefix(r) != ef:
                    errors.append(("compress", t, k, r, er))
                    continue
                src2 = make_sg(blk, segs, shuffle_seed=k)
                dst2 = make_sg(b"", [4096] * (-(-cap // 4096) or 1), capacity=cap)
                oracle_ref.compress_sg(src2, dst2)
                if src.it.as_tuple() != src2.it.as_tuple() or dst.it.as_tuple() != dst2.it.as_tuple():
                    errors.append(("iterators", t, k))
                d = gpu.decompress_safe(ef, n)
                if d != (n, blk):
                    errors.append(("decompress", t, k, d[0]))
                if k % 7 == 3 and len(ef) > 2:  # a truncated frame: the reference's error code
                    want = oracle_ref.decompress(ef[:len(ef) // 2], n)[0]
                    got = gpu.decompress_safe(ef[:len(ef) // 2], n)[0]
                    if got != want:
                        errors.append(("code", t, k, got, want))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(("exception", t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:5]


# ---------------------------------------------------------------------------
# BASELINE configurations at full size: every frame and every decode
# ---------------------------------------------------------------------------

def _full_size(gpu, host, lens, bs, cls):
    """Device-resident compress + decompress of equal-stride blocks, then
    every frame against the oracle's and every decode against the input."""
    import torch
    n = len(lens)
    lens = np.asarray(lens, dtype=np.int64)
    offs = np.arange(n, dtype=np.int64) * bs
    caps = lens + lens // 255 + 16
    slot = (bs + bs // 255 + 16 + 64 + 15) // 16 * 16
    doffs = np.arange(n, dtype=np.int64) * slot
    dev = torch.device("cuda")
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).to(dev)
    d_src = torch.from_numpy(host).to(dev)
    d_dst = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    ret = torch.zeros(n, dtype=torch.int32, device=dev)
    gpu.compress_batch_dev(d_src, t(offs, np.int64), t(lens, np.int32), t(np.full(n, cls), np.uint8),
                           d_dst, t(doffs, np.int64), t(caps, np.int32), ret, max_len=bs)
    d_out = torch.zeros(n * bs + 64, dtype=torch.uint8, device=dev)
    dret = torch.zeros(n, dtype=torch.int32, device=dev)
    gpu.decompress_batch_dev(d_dst, t(doffs, np.int64), ret, d_out, t(offs, np.int64), t(lens, np.int32),
                             dret)
    torch.cuda.synchronize()
    g_ret, g_dst = ret.cpu().numpy(), d_dst.cpu().numpy()
    assert (dret.cpu().numpy() == lens).all()
    U = int(lens.sum())
    assert torch.equal(d_out[:U], d_src[:U])
    del d_out, d_src
    L = oracle_ref.load()
    c_out = np.zeros(n * slot, np.uint8)
    c_ret = np.zeros(n, np.int32)
    # named arrays: a temporary's buffer could be freed before the C call reads it
    a_off, a_len = offs.astype(np.uint64), lens.astype(np.uint32)
    a_tt, a_doff, a_cap = np.full(n, cls, np.uint8), doffs.astype(np.uint64), caps.astype(np.uint32)
    L.oracle_compress_linear_batch(host.ctypes.data, a_off.ctypes.data, a_len.ctypes.data,
                                   a_tt.ctypes.data, c_out.ctypes.data, a_doff.ctypes.data,
                                   a_cap.ctypes.data, c_ret.ctypes.data, n, 16)
    assert (g_ret == c_ret).all(), np.flatnonzero(g_ret != c_ret)[:10]
    # every frame's bytes: mask the slots' tails and compare whole buffers
    used = np.zeros(n * slot, dtype=bool).reshape(n, slot)
    used[np.arange(slot)[None, :] < g_ret[:, None]] = True
    used = used.reshape(-1)
    bad = np.flatnonzero((g_dst != c_out) & used)
    assert bad.size == 0, f"first differing frame {bad[0] // slot}"


@pytest.mark.parametrize("name", ["silesia64k", "sg512", "fio4k", "text256k"])
def test_full_size_every_frame(gpu, name):
    """configs[1..4] at BASELINE's sizes: 3234 x 64 KiB byU16 (Silesia-proxy),
    3234 x 64 KiB byU32 (the 128 x 512 B layout's class), 262144 x 4 KiB
    (1 GiB fio pattern), 3815 x 256 KiB (10^9 B of text, last block
    182,784 B)."""
    bs, cls, n, total = {"silesia64k": (65536, BYU16, 3234, None), "sg512": (65536, BYU32, 3234, None),
                         "fio4k": (4096, BYU16, 262144, None),
                         "text256k": (262144, BYU32, 3815, 10**9)}[name]
    total = total or n * bs
    host = np.zeros(n * bs, np.uint8)
    if name == "fio4k":
        host[:total] = corpus.fio_pattern(total, 0xF10)
    elif name == "text256k":
        host[:total] = corpus.text_proxy(total, 0x7E57)
    else:
        host[:total] = corpus.silesia_proxy(total, 0x5157)
    lens = np.full(n, bs, np.int64)
    lens[-1] = total - (n - 1) * bs
    _full_size(gpu, host, lens, bs, cls)


def test_full_size_sg512_layout_every_frame(gpu):
    """configs[3] in its own SG layout at full size: the 3234 Silesia-proxy
    blocks of 64 KiB, each a list of 128 bio_vecs of 512 B at random in-page
    offsets (pages in shuffled order), through lz4e_compress_sg_batch (host
    gather, one launch, scatter into 1000-byte destination segments).  Every
    frame and both iterators' post-state equal oracle_compress_sg's, the
    reference's per-access SG walk (lz4e_compress.c:184-211 class rules,
    lz4e_defs.h:352-585 accessors)."""
    bs, n, seg = 65536, 3234, 512
    data = corpus.silesia_proxy(n * bs, 0x5157)
    rng = np.random.default_rng(0x512)
    cap = compress_bound(bs)
    pairs, offs_all = [], []
    for i in range(n):
        offs = [int(x) for x in rng.integers(0, 4096, bs // seg)]
        offs_all.append(offs)
        src = make_sg(data[i * bs:(i + 1) * bs].tobytes(), [seg] * (bs // seg), offsets=offs,
                      shuffle_seed=i)
        dst = make_sg(b"", [1000] * (-(-cap // 1000)), capacity=cap)
        pairs.append((src, dst))
    assert all(gpu.table_type(s) == BYU32 for s, _ in pairs[:8])
    rets = gpu.compress_sg_batch(pairs)
    bad = []
    for i, ((s, d), r) in enumerate(zip(pairs, rets)):
        # the oracle walks the same source pages from the start iterator
        s.it.bi_size, s_after = bs, s.it.as_tuple()
        s.it.bi_idx, s.it.bi_bvec_done = 0, 0
        d2 = make_sg(b"", [1000] * (-(-cap // 1000)), capacity=cap)
        er = oracle_ref.compress_sg(s, d2)
        if r != er or d.read_prefix(r) != d2.read_prefix(er) or s_after != s.it.as_tuple() or \
                d.it.as_tuple() != d2.it.as_tuple():
            bad.append(i)
    assert not bad, f"{len(bad)} frames differ, first {bad[:5]}"


@pytest.mark.parametrize("kind", ["mixed", "text", "runs", "ints", "random", "small_alpha", "fio"])
def test_decompress_pipelined_vs_wave_decoder(gpu, kind):
    """The four decoders on the same frames -- the pipelined 4-wave decoder,
    the one-wave decoder, its LDS form and the group decoder -- valid frames,
    exact and spare capacities, and corrupted ones: identical values and
    bytes, all equal to the oracle's."""
    rng = np.random.default_rng(zlib.crc32(kind.encode()))
    data = _corpus(kind, 1 << 20, 31)
    frames, caps, want = [], [], []
    for i in range(48):
        n = int(rng.choice([0, 1, 13, 100, 4096, 20000, 65536, int(rng.integers(1, 65537))]))
        s0 = int(rng.integers(0, data.size - n + 1))
        blk = data[s0:s0 + n].tobytes()
        f = oracle_ref.compress(blk, BYU16)[1]
        mode = i % 6
        cap = n
        if mode == 1:
            cap = min(65536, n + int(rng.integers(1, 200)))
        elif mode == 2 and len(f) > 2:
            f = f[:int(rng.integers(1, len(f)))]
        elif mode == 3 and len(f) > 0:
            fb = bytearray(f)
            for _ in range(3):
                fb[int(rng.integers(0, len(fb)))] ^= 1 << int(rng.integers(0, 8))
            f = bytes(fb)
        elif mode == 4:
            cap = max(0, n - int(rng.integers(1, 64)))
        frames.append(f)
        caps.append(cap)
        want.append(oracle_ref.decompress(f, cap))
    r_wg, o_wg = _gpu_decompress(gpu, frames, caps, mode=DEC_PIPE)
    r_wv, o_wv = _gpu_decompress(gpu, frames, caps, mode=DEC_WAVE)
    r_sm, o_sm = _gpu_decompress(gpu, frames, caps, mode=DEC_SMALL)
    r_gp, o_gp = _gpu_decompress(gpu, frames, caps, mode=DEC_GROUP)
    for i, (er, eb) in enumerate(want):
        assert r_wg[i] == er == r_wv[i] == r_sm[i] == r_gp[i], \
            (i, r_wg[i], er, r_wv[i], r_sm[i], r_gp[i])
        if er >= 0:
            assert o_wg[i] == eb == o_wv[i] == o_sm[i] == o_gp[i], i


# ---------------------------------------------------------------------------
# dictionary mode: LZ4E extension of the reference's
# stubbed dict path, checked against the oracle's restatement (parity
# unpinned: the reference never runs this path)
# ---------------------------------------------------------------------------

DICT_SIZES = [0, 5, 8, 100, 4096, 65536, 100000]


def test_dict_compress_via_entry_point(gpu):
    """LZ4E_compress_usingDict through bio_vec layouts (4 KiB and 512 B
    segments, mid-segment starts) equals the oracle; the frame decodes with
    the dictionary."""
    rng = np.random.default_rng(21)
    pool = _corpus("mixed", 1 << 21, 21).tobytes()
    for i in range(28):
        dsize = DICT_SIZES[i % len(DICT_SIZES)]
        n = int(rng.choice([0, 12, 13, 1000, 4096, 30000, 65536]))
        s0 = int(rng.integers(dsize, len(pool) - n))
        dic, blk = pool[s0 - dsize:s0], pool[s0:s0 + n]
        seg = [4096, 512][i % 2]
        segs = [min(seg, n - j) for j in range(0, n, seg)] or [16]
        src = make_sg(blk, segs, shuffle_seed=i)
        cap = compress_bound(n)
        dst = make_sg(b"", [4096] * (-(-cap // 4096) or 1), capacity=cap)
        r = gpu.compress_using_dict(src, dst, dic)
        er, ef = oracle_ref.compress_dict(blk, dic)
        assert r == er, (i, n, dsize)
        got = dst.read_prefix(r)
        assert got == ef, (i, n, dsize)
        assert oracle_ref.decompress_dict(got, n, dic) == (n, blk)


def test_dict_compress_sg_batch(gpu):
    rng = np.random.default_rng(22)
    pool = _corpus("text", 1 << 20, 22).tobytes()
    pairs, dicts, want = [], [], []
    for i in range(20):
        dsize = DICT_SIZES[i % len(DICT_SIZES)]
        n = int(rng.integers(13, 65537))
        s0 = int(rng.integers(dsize, len(pool) - n))
        dic, blk = pool[s0 - dsize:s0], pool[s0:s0 + n]
        src = make_sg(blk, [min(4096, n - j) for j in range(0, n, 4096)])
        cap = compress_bound(n)
        dst = make_sg(b"", [4096] * (-(-cap // 4096)), capacity=cap)
        pairs.append((src, dst))
        dicts.append(dic)
        want.append(oracle_ref.compress_dict(blk, dic))
    rets = gpu.compress_sg_batch_dict(pairs, dicts)
    for i, (er, ef) in enumerate(want):
        assert rets[i] == er
        assert pairs[i][1].read_prefix(rets[i]) == ef


@pytest.mark.parametrize("big", [False, True], ids=["wave", "pipe"])
def test_dict_decompress_values_and_codes(gpu, big):
    """LZ4E_decompress_safe_usingDict / lz4e_decompress_batch_dict on valid
    frames, short dictionaries, truncations and bit flips: values, error
    codes and bytes equal the oracle's restatement of the extDict branches
    (lz4e_decompress.c:299-302, 339-378).  Batches of small blocks decode on
    the one-wave decoder, batches with 64 KiB blocks on the pipelined one."""
    rng = np.random.default_rng(23 + big)
    pool = _corpus("mixed", 1 << 21, 23).tobytes()
    frames, caps, dicts, want = [], [], [], []
    for i in range(48):
        dsize = DICT_SIZES[i % len(DICT_SIZES)]
        n = int(rng.choice([65536, 40000])) if big and i % 3 == 0 else int(rng.integers(13, 12000))
        s0 = int(rng.integers(dsize, len(pool) - n))
        dic, blk = pool[s0 - dsize:s0], pool[s0:s0 + n]
        f = oracle_ref.compress_dict(blk, dic)[1]
        mode = i % 5
        cap = n
        if mode == 1 and len(dic) > 20:
            dic = dic[int(rng.integers(1, len(dic) - 8)):]  # a shorter dictionary
        elif mode == 2 and len(f) > 2:
            f = f[:int(rng.integers(1, len(f)))]
        elif mode == 3 and len(f) > 0:
            fb = bytearray(f)
            for _ in range(3):
                fb[int(rng.integers(0, len(fb)))] ^= 1 << int(rng.integers(0, 8))
            f = bytes(fb)
        elif mode == 4:
            cap = max(0, n - int(rng.integers(1, 64)))
        frames.append(f)
        caps.append(cap)
        dicts.append(dic)
        want.append(oracle_ref.decompress_dict(f, cap, dic))
    got = gpu.decompress_batch_dict(frames, caps, dicts)
    for i, (er, eb) in enumerate(want):
        assert got[i][0] == er, (i, got[i][0], er)
        if er >= 0:
            assert got[i][1] == eb, i
    # the single-call entry point on a few of them
    for i in range(0, 48, 7):
        assert gpu.decompress_safe_using_dict(frames[i], caps[i], dicts[i]) == want[i]


@pytest.mark.parametrize("dec", [DEC_GROUP, DEC_GROUP_NB, DEC_WAVE], ids=["group", "group_nobail", "wave"])
def test_dict_decompress_forced_decoders(gpu, dec):
    """A dictionary batch of small blocks through a forced decoder
    (lz4e_debug_decompress_dict): the group decoder with and without its
    hand-over, and the one-wave decoder.  Blocks open with a repeat of the
    dictionary's tail, so matches start in the dictionary and cross into the
    block; periods 2..40 exercise the group's period and doubling copies.
    Valid frames, truncations, flips and short capacities: values and bytes
    equal the oracle's restatement of the extDict branches
    (lz4e_decompress.c:299-302, 339-378)."""
    import torch
    rng = np.random.default_rng(77 + dec)
    pool = _corpus("mixed", 1 << 20, 29).tobytes()
    frames, caps, dicts, want = [], [], [], []
    for i in range(96):
        dsize = DICT_SIZES[i % len(DICT_SIZES)]
        s0 = int(rng.integers(dsize, len(pool) - 5000))
        dic = pool[s0 - dsize:s0]
        per = bytearray()
        for period in range(2 + i % 3, 41, 3):
            unit = rng.integers(0, 256, period, dtype=np.uint8).tobytes()
            per += rng.integers(0, 256, 23, dtype=np.uint8).tobytes() + (unit * 9)[:period * int(rng.integers(1, 8))]
        blk = ((dic[-200:] * 3)[:int(rng.integers(20, 600))] if dic else b"") + bytes(per) + pool[s0:s0 + 300]
        blk = blk[:4096]
        f = oracle_ref.compress_dict(blk, dic)[1]
        cap = len(blk)
        if i % 5 == 2 and len(f) > 2:
            f = f[:int(rng.integers(1, len(f)))]
        elif i % 5 == 3 and len(f) > 0:
            fb = bytearray(f)
            for _ in range(3):
                fb[int(rng.integers(0, len(fb)))] ^= 1 << int(rng.integers(0, 8))
            f = bytes(fb)
        elif i % 5 == 4:
            cap = max(0, len(blk) - int(rng.integers(1, 64)))
        frames.append(f)
        caps.append(cap)
        dicts.append(dic)
        want.append(oracle_ref.decompress_dict(f, cap, dic))
    # device layout: [dictionary | output capacity] per block, frames packed
    dev = torch.device("cuda")
    n = len(frames)
    soffs = np.concatenate([[0], np.cumsum([(len(f) + 15) // 16 * 16 for f in frames])[:-1]]).astype(np.int64)
    src = np.zeros(int(soffs[-1]) + len(frames[-1]) + 16, np.uint8)
    for i, f in enumerate(frames):
        src[soffs[i]:soffs[i] + len(f)] = np.frombuffer(f, np.uint8)
    doffs, pos = [], 0
    for i in range(n):
        pos += (len(dicts[i]) + 15) // 16 * 16
        doffs.append(pos)
        pos += (max(caps[i], 1) + 79) // 16 * 16
    out = np.zeros(pos + 64, np.uint8)
    for i in range(n):
        if dicts[i]:
            out[doffs[i] - len(dicts[i]):doffs[i]] = np.frombuffer(dicts[i], np.uint8)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).to(dev)
    d_out = t(out, np.uint8)
    ret = torch.full((n,), -7777, dtype=torch.int32, device=dev)
    L = gpu.lib()
    P = ctypes.c_void_p
    L.lz4e_debug_decompress_dict.argtypes = [P] * 7 + [ctypes.c_uint32, ctypes.c_uint32, P, P, ctypes.c_uint32]
    a = [t(src, np.uint8), t(soffs, np.int64), t([len(f) for f in frames], np.int32), t(doffs, np.int64),
         t(caps, np.int32), t([len(d) for d in dicts], np.int32)]
    assert L.lz4e_debug_decompress_dict(a[0].data_ptr(), a[1].data_ptr(), a[2].data_ptr(), d_out.data_ptr(),
                                        a[3].data_ptr(), a[4].data_ptr(), ret.data_ptr(), n, max(caps),
                                        a[5].data_ptr(), None, dec) == 0
    torch.cuda.synchronize()
    r = ret.cpu().numpy()
    o = d_out.cpu().numpy()
    for i, (er, eb) in enumerate(want):
        assert r[i] == er, (i, r[i], er)
        if er >= 0:
            assert o[doffs[i]:doffs[i] + er].tobytes() == eb, i


def test_dict_streams_device_resident(gpu):
    """Streams of 64 KiB blocks where block k's dictionary is block k-1
    (dict_len bytes right before the block in HBM): one compress launch over
    every block of every stream (blocks are independent given their
    dictionaries), frames equal the oracle's; then decode block index by block
    index across the streams, each block's dictionary being the previous
    block's decoded output in place -- the stream round trips."""
    import torch
    amd = gpu
    S, K, bs = 6, 5, 65536
    dev = torch.device("cuda")
    host = _corpus("mixed", S * K * bs, 24)
    src = torch.from_numpy(host).to(dev)
    n = S * K
    offs = np.arange(n, dtype=np.int64) * bs                  # stream s block k at (s*K + k) * bs
    dlen = np.array([min(k * bs, 65536) for s in range(S) for k in range(K)], np.int64)
    cap = bs + bs // 255 + 16
    slot = (cap + 64 + 15) // 16 * 16
    doffs = np.arange(n, dtype=np.int64) * slot
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).to(dev)
    dst = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    ret = torch.zeros(n, dtype=torch.int32, device=dev)
    L = amd.lib()
    ptr = lambda x: x.data_ptr()
    d_off, d_len, d_tt = t(offs, np.int64), t(np.full(n, bs), np.int32), t(np.full(n, BYU32), np.uint8)
    d_doff, d_cap, d_dl = t(doffs, np.int64), t(np.full(n, cap), np.int32), t(dlen, np.int32)
    assert L.lz4e_compress_batch_dev_dict(ptr(src), ptr(d_off), ptr(d_len), ptr(d_tt), ptr(dst),
                                          ptr(d_doff), ptr(d_cap), ptr(ret), None, n, bs,
                                          ptr(d_dl), None) == 0
    torch.cuda.synchronize()
    r = ret.cpu().numpy()
    d = dst.cpu().numpy()
    for i in range(n):
        k = i % K
        blk = host[i * bs:(i + 1) * bs].tobytes()
        dic = host[i * bs - int(dlen[i]):i * bs].tobytes() if k else b""
        er, ef = oracle_ref.compress_dict(blk, dic)
        assert r[i] == er and d[doffs[i]:doffs[i] + r[i]].tobytes() == ef, i
    # decode: launch k decodes block k of every stream into the stream's
    # contiguous output, after block k-1 (its dictionary)
    out = torch.zeros(n * bs + 64, dtype=torch.uint8, device=dev)
    dret = torch.full((n,), -9, dtype=torch.int32, device=dev)
    for k in range(K):
        idx = np.array([s * K + k for s in range(S)])
        a_soff, a_slen = t(doffs[idx], np.int64), t(r[idx], np.int32)
        a_doff, a_cap, a_dl = t(offs[idx], np.int64), t(np.full(S, bs), np.int32), t(dlen[idx], np.int32)
        rr = torch.zeros(S, dtype=torch.int32, device=dev)
        assert L.lz4e_decompress_batch_dev_dict(ptr(dst), ptr(a_soff), ptr(a_slen), ptr(out),
                                                ptr(a_doff), ptr(a_cap), ptr(rr), S, bs,
                                                ptr(a_dl), None) == 0
        dret[torch.from_numpy(idx).to(dev)] = rr
    torch.cuda.synchronize()
    assert (dret.cpu().numpy() == bs).all()
    assert np.array_equal(out[:n * bs].cpu().numpy(), host)


# ---------------------------------------------------------------------------
# launch order (lz4e_order.h): a schedule, never a result
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("nblocks,bs", [(1100, 65536), (3, 65536), (1025, 16384)])
def test_launch_order_does_not_change_results(gpu, nblocks, bs):
    """Heavy-first launch order only decides which workgroup handles which
    block: frames, iterator post-state, decoded bytes and return values are
    identical in block order and in launch order (forced on for batches
    below the size thresholds too), and equal the oracle's."""
    L = gpu.lib()
    L.lz4e_debug_set_launch_order.argtypes = [ctypes.c_int, ctypes.c_int]
    data = _corpus("mixed", nblocks * bs, 23)
    blocks = [data[i * bs:(i + 1) * bs].tobytes() for i in range(nblocks)]
    # a few ragged blocks (the weight sample clamps, tiny blocks weigh 0)
    blocks[1] = blocks[1][:700]
    blocks[-1] = blocks[-1][:bs - 5]
    ttypes = [BYU16] * nblocks
    runs = {}
    try:
        for mode in (0, 2):
            L.lz4e_debug_set_launch_order(mode, mode)
            r, frames, aux = _gpu_compress(gpu, blocks, ttypes)
            dr, dec = _gpu_decompress(gpu, frames, [bs] * nblocks, max_cap=bs)
            runs[mode] = (r, frames, aux, dr, dec)
    finally:
        L.lz4e_debug_set_launch_order(-1, -1)
    (r0, f0, a0, dr0, d0), (r2, f2, a2, dr2, d2) = runs[0], runs[2]
    assert (r0 == r2).all() and f0 == f2 and (a0 == a2).all()
    assert (dr0 == dr2).all() and d0 == d2
    for i in range(0, nblocks, max(1, nblocks // 64)):
        er, ef, efs, elr = oracle_ref.compress(blocks[i], BYU16)
        assert (r2[i], f2[i], a2[i][0], a2[i][1]) == (er, ef, efs, elr), i
        assert dr2[i] == len(blocks[i]) and d2[i] == blocks[i], i
