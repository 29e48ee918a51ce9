"""The kernels' own sources on the CPU, under ASan + UBSan.

tools/emu compiles lz4-sgori_amd/csrc/lz4e_compress.hip and
lz4e_decompress.hip unmodified as host C++ with every lane a thread, together
with the product's own csrc/lz4e_wave.h (built with -DLZ4E_EMU; the amdgcn
builtins it uses -- DPP row shifts, ds_(b)permute, v_perm, ballots -- are
emulated in tools/emu/include/hip/hip_runtime.h).  Workgroups of several
waves run as 64 threads per wave: the pipelined decoder's parser and copiers
meet through its LDS counters as host atomics.  It is the only CPU build of
the kernels, so it is where out-of-bounds reads and writes get caught before
they reach a GPU.  Each block's frame and iterator post-state, and each
decode's value and bytes, must equal the oracle's.

UBSan's alignment check is off: the kernel's unaligned dword loads are legal
on gfx950 (global loads need no alignment) and are emulated as plain loads.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle_ref
from lz4e_amd import BYU16, BYU32, BYU64, corpus

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CXX = "/opt/rocm/llvm/bin/clang++"


def _build_emu(tmp_path_factory, *extra):
    if not os.path.exists(CXX):
        pytest.skip("no clang++ for the emulator")
    b = tmp_path_factory.mktemp("emu")
    env = dict(os.environ, EMU_EXE="1", EMU_BUILD=str(b), CXX=CXX)
    subprocess.run(["bash", os.path.join(REPO, "tools", "emu", "build.sh"),
                    "-fsanitize=address,undefined", "-fno-sanitize=alignment",
                    "-fno-sanitize-recover=all", *extra], check=True, env=env, capture_output=True)
    exe = b / "emu_main"
    assert exe.exists()
    return b, str(exe)


@pytest.fixture(scope="session")
def emu_exe(tmp_path_factory):
    b, exe = _build_emu(tmp_path_factory)
    yield exe
    shutil.rmtree(b, ignore_errors=True)


@pytest.fixture(scope="session")
def emu_exe_vecext(tmp_path_factory):
    """The decoder built with the pipelined decoder's vector length-extension
    scan (InWindow::ext_stop) in the one-wave parse."""
    b, exe = _build_emu(tmp_path_factory, "-DLZ4E_ONEWAVE_VEC_EXT=true")
    yield exe
    shutil.rmtree(b, ignore_errors=True)


def _block(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "text":
        return corpus.text_proxy(n, seed)
    if kind == "records":
        return corpus._records(n, rng)
    if kind == "ints":
        return corpus._int_table(n, rng)
    if kind == "runs":
        return corpus._runs(n, rng)
    if kind == "small_alpha":
        return rng.integers(0, 3, n, dtype=np.uint8)
    return rng.integers(0, 256, n, dtype=np.uint8)


CASES = [("text", 4096, BYU16), ("records", 16384, BYU16), ("ints", 8192, BYU32),
         ("runs", 65536, BYU32), ("random", 20000, BYU32), ("small_alpha", 6000, BYU16),
         ("text", 30000, BYU64), ("text", 12, BYU16), ("text", 13, BYU16), ("text", 0, BYU16),
         ("records", 32768, BYU16),
         # blocks of <= 4 KiB: staged input, narrow tables (packed byU16, u16 byU32/byU64)
         ("small_alpha", 4096, BYU16), ("ints", 4096, BYU16), ("runs", 4000, BYU16),
         ("text", 4096, BYU32), ("ints", 3000, BYU64), ("random", 4096, BYU16)]


@pytest.mark.parametrize("kind,n,cls", CASES, ids=[f"{k}-{n}-{c}" for k, n, c in CASES])
def test_emulated_kernel_sanitized(emu_exe, tmp_path, kind, n, cls):
    data = _block(kind, n, 11 + n).tobytes()
    blk, frame = tmp_path / "blk.bin", tmp_path / "frame.bin"
    blk.write_bytes(data)
    out = subprocess.run([emu_exe, str(blk), str(cls), str(frame)], capture_output=True, text=True,
                         timeout=1200)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "ERROR: AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr
    _, r, _, fs, lr = out.stdout.split()
    er, ef, efs, elr = oracle_ref.compress(data, cls)
    assert int(r) == er
    assert frame.read_bytes() == ef
    assert (int(fs), int(lr)) == (efs, elr)


DICT_CASES = [("text", 4096, 4096), ("records", 16384, 65536), ("ints", 8192, 100000),
              ("text", 20000, 9), ("text", 20000, 5), ("random", 5000, 3000), ("text", 12, 4096)]


@pytest.mark.parametrize("kind,n,dsize", DICT_CASES, ids=[f"{k}-{n}-d{d}" for k, n, d in DICT_CASES])
def test_emulated_kernel_dictionary_sanitized(emu_exe, tmp_path, kind, n, dsize):
    """Dictionary mode (LZ4E extension, parity unpinned) through the kernel
    source: the dictionary preload, a parse starting after the dictionary and
    candidates inside it, under ASan + UBSan; frames equal the oracle's and
    decode back with the dictionary."""
    data = _block(kind, n + dsize, 7 + n).tobytes()
    dic, blkb = data[:dsize], data[dsize:]
    blk, frame, dct = tmp_path / "blk.bin", tmp_path / "frame.bin", tmp_path / "dict.bin"
    blk.write_bytes(blkb)
    dct.write_bytes(dic)
    out = subprocess.run([emu_exe, str(blk), str(BYU32), str(frame), str(dct)], capture_output=True,
                         text=True, timeout=1200)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "ERROR: AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr
    r = int(out.stdout.split()[1])
    er, ef = oracle_ref.compress_dict(blkb, dic)
    assert r == er
    assert frame.read_bytes() == ef
    assert oracle_ref.decompress_dict(ef, n, dic) == (n, blkb)


# ---------------------------------------------------------------------------
# the one-wave decoder's source on the CPU (emu_main -d), ASan + UBSan: the
# output buffer is exactly [dictionary | capacity], so a read before the
# dictionary or a write past the capacity is caught
# ---------------------------------------------------------------------------

def _emu_decode(exe, tmp_path, frame, cap, dic=b"", flag="-d"):
    f, o, d = tmp_path / "f.bin", tmp_path / "o.bin", tmp_path / "d.bin"
    f.write_bytes(frame)
    d.write_bytes(dic)
    if o.exists():
        o.unlink()
    out = subprocess.run([exe, flag, str(f), str(cap), str(o), str(d)], capture_output=True, text=True,
                         timeout=1200)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "ERROR: AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr
    r = int(out.stdout.split()[1])
    return r, (o.read_bytes() if r > 0 else b"")


DEC_CASES = [(k, m) for k in ("text", "records", "runs", "small_alpha") for m in range(5)]


DEC_RUNS = [(k, m, "-d") for k, m in DEC_CASES]


@pytest.mark.parametrize("kind,mode,flag", DEC_RUNS, ids=[f"{k}-{m}-wave" for k, m, f in DEC_RUNS])
def test_emulated_decoder_sanitized(emu_exe, tmp_path, kind, mode, flag):
    """Valid frames (mode 0), truncations (1), bit flips (2), short capacity
    (3) and a dictionary (4; with a shortened dictionary on odd seeds): the
    decoder's values, error codes and bytes equal the oracle's."""
    rng = np.random.default_rng(100 + mode)
    for rep in range(3):
        n = int(rng.integers(13, 20000))
        data = _block(kind, n + 9000, 3 + rep + n).tobytes()
        dic, blk = (data[:9000], data[9000:]) if mode == 4 else (b"", data[:n])
        f = oracle_ref.compress_dict(blk, dic)[1] if mode == 4 else oracle_ref.compress(blk, BYU16)[1]
        cap = len(blk)
        if mode == 1:
            f = f[:int(rng.integers(1, len(f)))]
        elif mode == 2:
            fb = bytearray(f)
            for _ in range(3):
                fb[int(rng.integers(0, len(fb)))] ^= 1 << int(rng.integers(0, 8))
            f = bytes(fb)
        elif mode == 3:
            cap = max(0, cap - int(rng.integers(1, 40)))
        elif mode == 4 and rep % 2:
            dic = dic[int(rng.integers(1, len(dic) - 8)):]
        want = oracle_ref.decompress_dict(f, cap, dic)
        got = _emu_decode(emu_exe, tmp_path, f, cap, dic, flag)
        assert got[0] == want[0], (rep, got[0], want[0])
        if want[0] >= 0:
            assert got[1] == want[1], rep


SMALL_CASES = [(k, m) for k in ("text", "runs", "fio") for m in range(5)]


@pytest.mark.parametrize("kind,mode", SMALL_CASES, ids=[f"{k}-{m}" for k, m in SMALL_CASES])
def test_emulated_small_block_decoder_sanitized(emu_exe, tmp_path, kind, mode):
    """The one-wave decoder's LDS-output form (blocks of <= 4608 bytes, the
    whole output assembled in LDS, scalar-path sequences copied LDS to LDS):
    valid frames (mode 0), truncations (1), bit flips (2), short capacity (3)
    and a dictionary (4: such blocks take the HBM form) equal the oracle."""
    rng = np.random.default_rng(500 + mode)
    for rep in range(3):
        n = int(rng.choice([4096, int(rng.integers(13, 4609))]))
        if kind == "fio":  # fio-style 4 KiB buffers: long literal runs and long matches
            fio = corpus.fio_pattern(16 * 4096)
            data = fio[(rep + 2) * 4096 - 9000:][:n + 9000].tobytes()
        else:
            data = _block(kind, n + 9000, 11 + rep + n).tobytes()
        dic, blk = (data[:9000], data[9000:]) if mode == 4 else (b"", data[:n])
        f = oracle_ref.compress_dict(blk, dic)[1] if mode == 4 else oracle_ref.compress(blk, BYU16)[1]
        cap = len(blk) + (32 if rep == 1 else 0)
        if mode == 1:
            f = f[:int(rng.integers(1, len(f)))]
        elif mode == 2:
            fb = bytearray(f)
            for _ in range(3):
                fb[int(rng.integers(0, len(fb)))] ^= 1 << int(rng.integers(0, 8))
            f = bytes(fb)
        elif mode == 3:
            cap = max(0, len(blk) - int(rng.integers(1, 40)))
        want = oracle_ref.decompress_dict(f, cap, dic)
        got = _emu_decode(emu_exe, tmp_path, f, cap, dic, "-l")
        assert got[0] == want[0], (rep, got[0], want[0])
        if want[0] >= 0:
            assert got[1] == want[1], rep


LANE_CASES = [(k, m) for k in ("text", "fio", "random", "head") for m in range(5)]


@pytest.mark.parametrize("kind,mode", LANE_CASES, ids=[f"{k}-{m}" for k, m in LANE_CASES])
def test_emulated_lane_decoder_sanitized(emu_exe, tmp_path, kind, mode):
    """The block-per-group decoder (one block per 8-lane group, copies over
    the group) and its hand-over to
    the one-wave decoder: blocks that open with a short literal run go over
    at once (text), long-sequence blocks stay on their lane (fio, random),
    and "head" blocks (230 random bytes, 200 zeros, then text) go over
    mid-block at a sequence boundary.  Valid frames (mode 0), truncations (1), bit
    flips (2), short capacity (3) and a dictionary (4) equal the oracle."""
    rng = np.random.default_rng(700 + mode)
    for rep in range(3):
        n = int(rng.choice([4096, int(rng.integers(13, 12000))]))
        if kind == "fio":
            data = corpus.fio_pattern(16 * 4096)[(rep + 2) * 4096 - 9000:][:n + 9000].tobytes()
        elif kind == "head":
            t = _block("text", n + 9000, 5 + rep).tobytes()
            r = np.random.default_rng(rep).integers(0, 256, 230, dtype=np.uint8).tobytes() + bytes(200)
            data = t[:9000] + (r + t[9000:])[:n]
        else:
            data = _block(kind, n + 9000, 21 + rep + n).tobytes()
        dic, blk = (data[:9000], data[9000:]) if mode == 4 else (b"", data[9000:9000 + n] if kind == "head" else data[:n])
        f = oracle_ref.compress_dict(blk, dic)[1] if mode == 4 else oracle_ref.compress(blk, BYU16)[1]
        cap = len(blk)
        if mode == 1:
            f = f[:int(rng.integers(1, len(f)))]
        elif mode == 2:
            fb = bytearray(f)
            for _ in range(3):
                fb[int(rng.integers(0, len(fb)))] ^= 1 << int(rng.integers(0, 8))
            f = bytes(fb)
        elif mode == 3:
            cap = max(0, len(blk) - int(rng.integers(1, 40)))
        want = oracle_ref.decompress_dict(f, cap, dic)
        got = _emu_decode(emu_exe, tmp_path, f, cap, dic, "-g")
        assert got[0] == want[0], (rep, got[0], want[0])
        if want[0] >= 0:
            assert got[1] == want[1], rep


def _periodic_block(rng, periods, reps=(1, 2, 3, 17)):
    """Self-overlapping matches of every period in `periods` at lengths around
    1x-17x the period, separated by random bytes (the overlap-copy cases)."""
    parts = []
    for period in periods:
        for rep in reps:
            parts.append(rng.integers(0, 256, 37, dtype=np.uint8).tobytes())
            unit = rng.integers(0, 256, period, dtype=np.uint8).tobytes()
            parts.append((unit * (rep + 2))[:period * rep + int(rng.integers(0, period))])
    return b"".join(parts) + rng.integers(0, 256, 20, dtype=np.uint8).tobytes()


NOBAIL_CASES = [(k, m) for k in ("text", "fio", "head") for m in range(5)] + \
               [("periodic", 0), ("periodic", 3), ("periodic_dict", 0), ("periodic_dict", 1), ("periodic_dict", 4)]


@pytest.mark.parametrize("kind,mode", NOBAIL_CASES, ids=[f"{k}-{m}" for k, m in NOBAIL_CASES])
def test_emulated_group_decoder_no_handover(emu_exe, tmp_path, kind, mode):
    """The group decoder with its hand-over disabled (-G, kDecGroupNoBail):
    its own copies run on every block -- text and "head" blocks of short
    sequences that the hand-over would give away, the period-from-registers
    path for offsets 2-15, offset doubling from 16 on, and (periodic_dict)
    matches that start in the dictionary and run on into the block.  Valid
    frames (mode 0), truncations (1), bit flips (2), short capacity (3) and a
    shortened dictionary (4) equal the oracle."""
    rng = np.random.default_rng(900 + mode + 11 * len(kind))
    for rep in range(2):
        dic = b""
        if kind.startswith("periodic"):
            blk = _periodic_block(rng, range(2 + rep, 41, 2))
            if kind == "periodic_dict":
                dic = rng.integers(0, 256, 9000, dtype=np.uint8).tobytes()
                # the block opens with the dictionary's tail, repeated: its
                # first matches start in the dictionary and cross into the block
                blk = (dic[-300:] * 3)[:700] + dic[-40:] + blk
        else:
            n = int(rng.choice([4096, int(rng.integers(13, 12000))]))
            if kind == "fio":
                blk = corpus.fio_pattern(16 * 4096)[(rep + 2) * 4096:][:n].tobytes()
            elif kind == "head":
                t = _block("text", n, 5 + rep).tobytes()
                r = np.random.default_rng(rep).integers(0, 256, 230, dtype=np.uint8).tobytes() + bytes(200)
                blk = (r + t)[:n]
            else:
                blk = _block(kind, n, 21 + rep + n).tobytes()
        f = oracle_ref.compress_dict(blk, dic)[1] if dic else oracle_ref.compress(blk, BYU16)[1]
        cap = len(blk)
        if mode == 1:
            f = f[:int(rng.integers(1, len(f)))]
        elif mode == 2:
            fb = bytearray(f)
            for _ in range(3):
                fb[int(rng.integers(0, len(fb)))] ^= 1 << int(rng.integers(0, 8))
            f = bytes(fb)
        elif mode == 3:
            cap = max(0, len(blk) - int(rng.integers(1, 40)))
        elif mode == 4 and dic:
            dic = dic[int(rng.integers(1, 200)):]
        want = oracle_ref.decompress_dict(f, cap, dic)
        got = _emu_decode(emu_exe, tmp_path, f, cap, dic, "-G")
        assert got[0] == want[0], (rep, got[0], want[0])
        if want[0] >= 0:
            assert got[1] == want[1], rep


VEC_CASES = [(k, m) for k in ("random", "runs", "text") for m in range(4)]


@pytest.mark.parametrize("kind,mode", VEC_CASES, ids=[f"{k}-{m}" for k, m in VEC_CASES])
def test_emulated_decoder_vector_extension_scan(emu_exe_vecext, tmp_path, kind, mode):
    """The length-extension scan (one ballot per 256 window bytes instead of
    the reference's byte loop, lz4e_decompress.c:201-206, 319-326): values,
    error codes and bytes equal the oracle's on valid frames (mode 0),
    truncations (1), bit flips (2) and short capacity (3); random data gives
    literal runs with extensions of up to ~55 bytes, runs long match
    extensions."""
    rng = np.random.default_rng(300 + mode)
    for rep in range(2):
        n = int(rng.integers(4500, 14000))
        blk = _block(kind, n, 5 + rep + n).tobytes()
        f = oracle_ref.compress(blk, BYU16)[1]
        cap = len(blk)
        if mode == 1:
            f = f[:int(rng.integers(1, len(f)))]
        elif mode == 2:
            fb = bytearray(f)
            for _ in range(3):
                fb[int(rng.integers(0, len(fb)))] ^= 1 << int(rng.integers(0, 8))
            f = bytes(fb)
        elif mode == 3:
            cap = max(0, cap - int(rng.integers(1, 40)))
        want = oracle_ref.decompress_dict(f, cap, b"")
        got = _emu_decode(emu_exe_vecext, tmp_path, f, cap)
        assert got[0] == want[0], (rep, got[0], want[0])
        if want[0] >= 0:
            assert got[1] == want[1], rep


def test_emulated_decoder_vector_extension_truncated_in_run(emu_exe_vecext, tmp_path):
    """Frames cut inside and just after a literal-length extension run (the
    reference's end checks on the run, lz4e_decompress.c:197-206), and an
    extension run whose 255 bytes reach the frame end."""
    blk = _block("random", 12000, 77).tobytes()
    f = oracle_ref.compress(blk, BYU16)[1]
    ext = 1
    while f[ext] == 255:
        ext += 1
    cuts = sorted({1, 2, 3, ext - 1, ext, ext + 1, ext + 2, ext + 15, ext + 16, ext + 17, ext + 40})
    for k in cuts:
        ff = f[:k]
        want = oracle_ref.decompress_dict(ff, len(blk), b"")
        got = _emu_decode(emu_exe_vecext, tmp_path, ff, len(blk))
        assert got[0] == want[0], (k, got[0], want[0])
    ff = bytes([0xF0]) + b"\xff" * 300
    want = oracle_ref.decompress_dict(ff, 100000, b"")
    got = _emu_decode(emu_exe_vecext, tmp_path, ff, 100000)
    assert got[0] == want[0], (got[0], want[0])


# ---------------------------------------------------------------------------
# The pipelined decoder (decompress_pipe_kernel: one parser wave and three
# copier waves per block, LDS record ring, spans, progress counters as host
# atomics) on the emulator, under the same sanitizers.
# ---------------------------------------------------------------------------

def _emu_decode_pipe(exe, tmp_path, frame, cap, dic=b"", flag="-p"):
    f, o, d = tmp_path / "f.bin", tmp_path / "o.bin", tmp_path / "d.bin"
    f.write_bytes(frame)
    d.write_bytes(dic)
    if o.exists():
        o.unlink()
    out = subprocess.run([exe, flag, str(f), str(cap), str(o), str(d)], capture_output=True, text=True,
                         timeout=1200)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "ERROR: AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr
    lines = out.stdout.split("\n")
    r = int(lines[0].split()[1])
    return r, (o.read_bytes() if r > 0 else b""), lines[1]


PIPE_CASES = [(k, m) for k in ("text", "records", "ints", "runs") for m in range(5)] + [("random", 0)]


PIPE_RUNS = [(k, m, "-p") for k, m in PIPE_CASES]
_PN = {"-p": "pipe"}


@pytest.mark.parametrize("kind,mode,flag", PIPE_RUNS, ids=[f"{k}-{m}-{_PN[f]}" for k, m, f in PIPE_RUNS])
def test_emulated_pipe_decoder_sanitized(emu_exe, tmp_path, kind, mode, flag):
    """The 4-wave pipelined decoder (-p) on 16-64 KiB blocks: valid frames (mode 0), truncations (1), bit flips
    (2), short capacity (3) and a dictionary (4): values, error codes and
    bytes equal the oracle's (/root/reference/lz4e/lz4e_decompress.c:62-460
    restated)."""
    rng = np.random.default_rng(700 + mode + 17 * len(kind))
    n = int(rng.integers(16384, 65536))
    data = _block(kind, n + 9000, 31 + n).tobytes()
    dic, blk = (data[:9000], data[9000:]) if mode == 4 else (b"", data[:n])
    f = oracle_ref.compress_dict(blk, dic)[1] if mode == 4 else oracle_ref.compress(blk, BYU16)[1]
    cap = len(blk)
    if mode == 1:
        f = f[:int(rng.integers(1, len(f)))]
    elif mode == 2:
        fb = bytearray(f)
        for _ in range(3):
            fb[int(rng.integers(0, len(fb)))] ^= 1 << int(rng.integers(0, 8))
        f = bytes(fb)
    elif mode == 3:
        cap = max(0, cap - int(rng.integers(1, 40)))
    want = oracle_ref.decompress_dict(f, cap, dic)
    got = _emu_decode_pipe(emu_exe, tmp_path, f, cap, dic, flag)
    assert got[0] == want[0], (got[0], want[0])
    if want[0] >= 0:
        assert got[1] == want[1]


@pytest.fixture(scope="session")
def emu_exe_spin1(tmp_path_factory):
    """The decoders built with a watchdog limit of one sleep and no per-byte
    term: any wait that needs a second poll gives up (LZ4E_SPIN_MAX=1,
    LZ4E_SPIN_BYTES_SHIFT=31)."""
    b, exe = _build_emu(tmp_path_factory, "-DLZ4E_SPIN_MAX=1", "-DLZ4E_SPIN_BYTES_SHIFT=31")
    yield exe
    shutil.rmtree(b, ignore_errors=True)


@pytest.mark.parametrize("flag", ["-p"], ids=["pipe"])
def test_emulated_pipe_decoder_watchdog(emu_exe_spin1, tmp_path, flag):
    """A forced watchdog: every wave leaves its loop (the run ends), the
    block's value is LZ4E_DECODE_ABORTED -- even though the parser itself
    finished the parse -- and the host's reading of the batch
    (csrc/lz4e_results.h, used by every host entry point) fails the call
    with the watchdog named in lz4e_last_error's text."""
    blk = _block("text", 65536, 9).tobytes()
    f = oracle_ref.compress(blk, BYU16)[1]
    r, _, res = _emu_decode_pipe(emu_exe_spin1, tmp_path, f, len(blk), flag=flag)
    assert r == -2**31
    good, msg = res.split(" ", 2)[1:]
    assert int(good) == -1 and "watchdog" in msg and "LZ4E_DECODE_ABORTED" in msg
