#!/bin/bash
# Round 5 final build (group decoder): smoke, every -m gpu test, the default
# bench (all legs), the other workload lines, fio4k FETCH/WRITE, kernel stats.
tag=${1:-r05s}
o=gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 2 "$o/$name.log" | cut -c1-300 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -30 "$o/$name.log" >&2; exit $rc; fi; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step pytest 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 500 python -u bench.py
for w in fio4k sg512 text256k; do
  step bench_$w 420 python -u bench.py --workload $w --no-single-call
done
WORKLOADS=fio4k step pmc_fio 600 bash tools/pmc_workloads.sh $tag/pmcw
step prof_fio 300 rocprofv3 --kernel-trace --stats -T -d $o/prof_fio -o run --output-format csv -- python3 bench.py --workload fio4k --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-single-call --no-parity --no-strong --no-decompress-only
