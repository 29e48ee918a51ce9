"""Per-kernel duration summary from a rocprofv3 rocpd database (the format
this ROCm's rocprofv3 writes by default): name, calls, mean / min / max
microseconds, grid.  usage: python tools/rocpd_stats.py RESULTS.db [name filter]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = c.execute("select name, duration, grid_x, workgroup_x, vgpr_count, lds_size from kernels").fetchall()
agg = {}
for name, d, g, w, v, lds in rows:
    short = name.replace("void ", "").replace("lz4e::(anonymous namespace)::", "").split("(")[0]
    if flt not in short:
        continue
    agg.setdefault((short, g, w, v, lds), []).append(d / 1000.0)
for (n, g, w, v, lds), ds in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{n[:70]:70s} grid {g:8d} wg {w:4d} vgpr {v:4d} lds {lds:6d}: calls {len(ds):3d} "
          f"mean {sum(ds) / len(ds):9.1f} us  min {min(ds):9.1f}  max {max(ds):9.1f}")
try:
    mc = c.execute("select name, duration, size from memory_copies").fetchall()
except sqlite3.Error:
    mc = []
magg = {}
for name, d, sz in mc:
    magg.setdefault((name, sz), []).append(d / 1000.0)
for (n, sz), ds in sorted(magg.items(), key=lambda kv: -len(kv[1]))[:8]:
    print(f"copy {str(n)[:40]:40s} {sz:10d} B: calls {len(ds):4d} mean {sum(ds) / len(ds):8.1f} us")

