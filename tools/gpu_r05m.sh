#!/bin/bash
# Round 5: narrow hash tables for blocks of <= 4 KiB -- every -m gpu test,
# the fio4k line, the default bench, then the fio4k SQ counters.
tag=${1:-r05m}
o=gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 3 "$o/$name.log" | cut -c1-1500 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -30 "$o/$name.log" >&2; exit $rc; fi; }
step pytest 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench_fio4k 420 python -u bench.py --workload fio4k --no-single-call
step bench 400 python -u bench.py
BENCH_ARGS="--workload fio4k --no-decompress-only" step sqfio 600 bash tools/pmc_sq.sh r05m/sqfio
