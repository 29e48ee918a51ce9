"""The compress kernel's own source on the CPU, under ASan + UBSan.

tools/emu compiles lz4-sgori_amd/csrc/lz4e_compress.hip unmodified as host
C++ with every lane of the wave a thread (tools/emu/lz4e_wave.h stands in for
the wave primitives).  It is the only CPU build of the kernel, so it is where
out-of-bounds window / candidate / stripe reads get caught before they reach
a GPU.  Each block's frame and iterator post-state must equal the oracle's.

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


@pytest.fixture(scope="session")
def emu_exe(tmp_path_factory):
    if not os.path.exists(CXX):
        pytest.skip("no clang++ for the emulator")
    b = tmp_path_factory.mktemp("emu")
    env = dict(os.environ, EMU_EXE="1", EMU_BUILD=str(b), CXX=CXX)
    subprocess.run(["bash", os.path.join(REPO, "tools", "emu", "build.sh"),
                    "-fsanitize=address,undefined", "-fno-sanitize=alignment",
                    "-fno-sanitize-recover=all"], check=True, env=env, capture_output=True)
    exe = b / "emu_main"
    assert exe.exists()
    yield str(exe)
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
         ("records", 65536, BYU16)]


@pytest.mark.parametrize("kind,n,cls", CASES, ids=[f"{k}-{n}-{c}" for k, n, c in CASES])
def test_emulated_kernel_sanitized(emu_exe, tmp_path, kind, n, cls):
    data = _block(kind, n, 11 + n).tobytes()
    blk, frame = tmp_path / "blk.bin", tmp_path / "frame.bin"
    blk.write_bytes(data)
    out = subprocess.run([emu_exe, str(blk), str(cls), str(frame)], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "ERROR: AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr
    _, r, _, fs, lr = out.stdout.split()
    er, ef, efs, elr = oracle_ref.compress(data, cls)
    assert int(r) == er
    assert frame.read_bytes() == ef
    assert (int(fs), int(lr)) == (efs, elr)
