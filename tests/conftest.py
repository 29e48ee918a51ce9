"""pytest configuration: the `gpu` marker and shared fixtures.

`-m "not gpu"` runs the oracle-vs-golden tests, host logic and the C-ABI
load/symbol checks (no GPU).  `-m gpu` runs the parity tests proper: the HIP
path through the C ABI against the CPU oracle on the same seeded inputs.
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs the HIP kernels)")


@pytest.fixture(scope="session")
def oracle():
    import oracle_ref
    return oracle_ref.load()


@pytest.fixture(scope="session")
def amd():
    import lz4e_amd
    lz4e_amd.lib()
    return lz4e_amd


@pytest.fixture(scope="session")
def gpu(amd):
    if not amd.gpu_available():
        pytest.fail("gpu-marked test but the library cannot reach a gfx950: " + amd.last_error())
    return amd


@pytest.fixture(scope="session")
def test_files():
    d = os.path.join(REPO, "tests", "golden", "test_files")
    return {n: open(os.path.join(d, n), "rb").read() for n in ("01.txt", "02.txt", "03.jpg")}
