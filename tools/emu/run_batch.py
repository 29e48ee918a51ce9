"""Run test_compress_batch_vs_oracle's blocks through the lane emulator
(tools/emu/build/libemu.so) and compare each frame with the oracle.

usage: python tools/emu/run_batch.py KIND CLS [max_len_filter]"""
import ctypes
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "lz4-sgori_amd")]
import oracle_ref  # noqa
from lz4e_amd import corpus  # noqa


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
    if kind == "records":
        return corpus._records(n, rng)
    if kind == "small_alpha":
        return rng.integers(0, 3, n, dtype=np.uint8)
    return corpus.silesia_proxy(n, seed)


def emu_compress(blocks, ttypes, lib):
    n = len(blocks)
    lens = np.array([len(b) for b in blocks], dtype=np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum((lens.astype(np.int64) + 15) // 16 * 16)[:-1]
    src = np.zeros(int(offs[-1] + lens[-1]) + 16, dtype=np.uint8)
    for i, b in enumerate(blocks):
        src[int(offs[i]):int(offs[i]) + len(b)] = np.frombuffer(b, dtype=np.uint8)
    caps = (lens + lens // 255 + 16).astype(np.uint32)
    slot = caps.astype(np.int64) + 64
    doffs = np.zeros(n, dtype=np.uint64)
    doffs[1:] = np.cumsum((slot + 15) // 16 * 16)[:-1]
    dst = np.full(int(doffs[-1] + slot[-1]) + 16, 0xCD, dtype=np.uint8)  # canary
    ret = np.full(n, -7, dtype=np.int32)
    aux = np.zeros(2 * n, dtype=np.uint32)
    tt = np.asarray(ttypes, dtype=np.uint8)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    rc = lib.emu_compress_batch(P(src), P(offs), P(lens), P(tt), P(dst), P(doffs), P(caps), P(ret),
                                P(aux), n, int(lens.max()))
    assert rc == 0
    frames = [dst[int(doffs[i]):int(doffs[i]) + max(0, int(ret[i]))].tobytes() for i in range(n)]
    for i in range(n):  # nothing may be written past the frame (or the slot, on failure)
        end = int(doffs[i]) + (int(ret[i]) if ret[i] > 0 else 0)
        tail = dst[end:int(doffs[i]) + int(slot[i])]
        if ret[i] > 0 and (tail != 0xCD).any():
            print(f"  block {i}: bytes written past the frame end at +{int(np.argmax(tail != 0xCD))}")
    return ret, frames, aux.reshape(n, 2)


def main():
    kind, cls = sys.argv[1], int(sys.argv[2])
    only = int(sys.argv[3]) if len(sys.argv) > 3 else None
    lib = ctypes.CDLL(os.path.join(HERE, "build", "libemu.so"))
    rng = np.random.default_rng(zlib.crc32(f"{kind}-{cls}".encode()))
    data = _corpus(kind, 1 << 21, 17)
    lens = [int(x) for x in rng.choice([0, 1, 12, 13, 14, 100, 4096, 4097, 30000, 65535, 65536], size=48)]
    if cls == 3:
        lens += [65537, 131072, 200000]
    blocks = []
    for ln in lens:
        s = int(rng.integers(0, data.size - ln))
        blocks.append(data[s:s + ln].tobytes())
    idx = [i for i in range(len(blocks)) if only is None or len(blocks[i]) == only]
    bad = 0
    for i in idx:  # one block per launch: a crash names its block
        r, f, a = emu_compress([blocks[i]], [cls], lib)
        er, ef, efs, elr = oracle_ref.compress(blocks[i], cls)
        ok = r[0] == er and f[0] == ef and (a[0][0], a[0][1]) == (efs, elr)
        if not ok:
            bad += 1
            k = next((j for j in range(min(len(f[0]), len(ef))) if f[0][j] != ef[j]), None)
            print(f"block {i} len {len(blocks[i])}: ret {r[0]} vs {er}, first diff {k}, aux {tuple(a[0])} vs {(efs, elr)}", flush=True)
        else:
            print(f"block {i} len {len(blocks[i])}: ok", flush=True)
    print("bad", bad, "of", len(idx))


if __name__ == "__main__":
    main()
