#!/bin/bash
# Round 5 final build: smoke, every -m gpu test, the default bench (all legs),
# the other workload lines, rocprofv3 kernel stats + FETCH/WRITE, SQ counters.
tag=${1:-r05z}
o=gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 2 "$o/$name.log" | cut -c1-400 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -30 "$o/$name.log" >&2; exit $rc; fi; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step pytest 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 500 python -u bench.py
for w in fio4k sg512 text256k; do
  step bench_$w 420 python -u bench.py --workload $w --no-single-call
done
rm -rf gpurun_out/prof_r05
step prof 900 bash tools/profile.sh r05
cp $(find gpurun_out/prof_r05/trace -name "*kernel_stats.csv" | head -1) $o/kernel_stats.csv
python3 tools/pmc_summary.py gpurun_out/prof_r05 silesia64k $o/pmc_traffic.json > $o/pmc_summary.log 2>&1
step sq 700 bash tools/pmc_sq.sh $tag/sq
