"""(Experiment record, not collected by the suite: run it explicitly with
python -m pytest tools/bandexp/test_emulator_band.py.)

The band compressor's own source (tools/bandexp/lz4e_band.hip) on the CPU lane
emulator under ASan + UBSan: every frame, its size and the iterator
post-state words equal the oracle's (tools/emu/emu_band_main.cpp), on the
block kinds whose parses exercise each of its paths -- short chains (text),
long matches that end a pass (runs), sparse searches past the 66th probe
(random, jpeg), periodic puts (ints, records), the three table classes,
limited output and the sizes around LZ4E_MIN_LENGTH."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from lz4e_amd import BYU16, BYU32, BYU64, corpus

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CXX = "/opt/rocm/llvm/bin/clang++"


@pytest.fixture(scope="session")
def band_exe(tmp_path_factory):
    if not os.path.exists(CXX):
        pytest.skip("no clang++ for the emulator")
    b = tmp_path_factory.mktemp("emuband")
    exe = str(b / "emu_band_main")
    subprocess.run(["bash", os.path.join(REPO, "tools", "bandexp", "build_band.sh"), exe,
                    "-fsanitize=address,undefined", "-fno-sanitize=alignment", "-fno-sanitize-recover=all"],
                   check=True, capture_output=True)
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
    if kind == "fio":
        return corpus.fio_pattern(n, seed)
    if kind == "jpeg":
        with open(os.path.join(REPO, "tests", "golden", "test_files", "03.jpg"), "rb") as f:
            return np.frombuffer(f.read()[:n], np.uint8)
    if kind == "small_alpha":
        return rng.integers(0, 3, n, dtype=np.uint8)
    return rng.integers(0, 256, n, dtype=np.uint8)


CASES = [("text", 4096, BYU16, 0), ("text", 20000, BYU16, 0), ("records", 16384, BYU16, 0),
         ("ints", 8192, BYU32, 0), ("runs", 65536, BYU32, 0), ("random", 20000, BYU32, 0),
         ("jpeg", 16384, BYU16, 0), ("fio", 8192, BYU16, 0), ("small_alpha", 6000, BYU16, 0),
         ("text", 30000, BYU64, 0), ("text", 12, BYU16, 0), ("text", 13, BYU16, 0),
         ("text", 0, BYU16, 0), ("text", 40, BYU32, 0), ("text", 1100, BYU16, 0),
         ("text", 8192, BYU16, -2000), ("random", 4096, BYU16, -10), ("text", 4096, BYU32, -1)]


@pytest.mark.parametrize("kind,n,tt,capd", CASES, ids=[f"{k}-{n}-{t}-{c}" for k, n, t, c in CASES])
def test_emulated_band_compressor_sanitized(band_exe, tmp_path, kind, n, tt, capd):
    blk = _block(kind, n, 17 + n + tt).tobytes()[:n]
    assert len(blk) == n
    f = tmp_path / "blk.bin"
    f.write_bytes(blk)
    out = subprocess.run([band_exe, str(f), str(n), str(tt), "1", str(capd)], capture_output=True, text=True,
                         timeout=900)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "bad=0" in out.stdout
