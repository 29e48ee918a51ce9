"""Offline: compare saved GPU frames with the oracle, print the first
divergent sequence of each mismatching block."""
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "lz4-sgori_amd")]
import oracle_ref  # noqa


def seqs(f):
    i, pos, out = 0, 0, []
    while i < len(f):
        t = f[i]; i += 1
        L = t >> 4
        if L == 15:
            while True:
                b = f[i]; i += 1; L += b
                if b != 255: break
        lit_at = pos
        i += L; pos += L
        if i >= len(f):
            out.append((lit_at, L, None, None)); break
        off = f[i] | f[i + 1] << 8; i += 2
        M = t & 15
        if M == 15:
            while True:
                b = f[i]; i += 1; M += b
                if b != 255: break
        M += 4
        out.append((lit_at, L, off, M)); pos += M
    return out


if __name__ == "__main__":
    for g in sorted(glob.glob(os.path.join(REPO, "gpurun_out", "dbg", "*.gpu"))):
      base = g[:-4]
      cls = int(os.path.basename(base).split("_")[1])
      data = open(base + ".in", "rb").read()
      gf = open(g, "rb").read()
      er, ef, _, _ = oracle_ref.compress(data, cls)
      if gf == ef:
          continue
      a, b = seqs(gf), seqs(ef)
      k = next((j for j in range(min(len(a), len(b))) if a[j] != b[j]), None)
      print(os.path.basename(base), len(data), "gpu", len(gf), "ref", len(ef), "first diff seq", k)
      if k is not None:
          for j in range(max(0, k - 2), min(k + 3, len(a), len(b))):
              print("   ", j, "gpu", a[j], "ref", b[j])
