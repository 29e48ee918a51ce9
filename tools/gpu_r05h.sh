#!/bin/bash
# Round 5 profiles: workload lines, rocprofv3 kernel stats + FETCH/WRITE of the
# default bench, SQ counters of the band experiment (u16 build).
tag=${1:-r05h}
o=gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 1 "$o/$name.log" | cut -c1-400 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -20 "$o/$name.log" >&2; exit $rc; fi; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for w in fio4k sg512 text256k; do
  step bench_$w 420 python -u bench.py --workload $w --no-single-call
done
step prof 900 bash tools/profile.sh r05
find gpurun_out/prof_r05 -name "*kernel_stats.csv" -exec cp {} $o/kernel_stats.csv \;
step band_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -T -d $o/band_sq -o run --output-format csv -- python3 tools/bandexp/bandstamps.py silesia 256
