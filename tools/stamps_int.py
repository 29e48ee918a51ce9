"""Diagnostic: compress phase cycles (stamped build) on integer-table blocks,
the slowest class of the Silesia-proxy (4-byte and 8-byte little-endian
counters with small increments, 64 KiB blocks, byU16)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import stamps  # noqa: E402

if __name__ == "__main__":
    rng = np.random.default_rng(5)
    k = 256 * 65536 // 4
    v4 = (np.uint64(12345) + np.cumsum(rng.integers(0, 64, size=k)).astype(np.uint64)) & np.uint64(0xFFFFFFFF)
    stamps.run("int4_64k", np.frombuffer(v4.astype("<u4").tobytes(), dtype=np.uint8).copy(), 65536, 1, "")
    v8 = np.uint64(12345) + np.cumsum(rng.integers(0, 64, size=k // 2)).astype(np.uint64)
    stamps.run("int8_64k", np.frombuffer(v8.astype("<u8").tobytes(), dtype=np.uint8).copy(), 65536, 1, "")
