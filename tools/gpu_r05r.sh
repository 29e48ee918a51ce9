#!/bin/bash
# Round 5: the group decoder as auto mode's small-block decoder -- every -m gpu
# test, decoders side by side (thresholds), fio4k and default lines.
o=gpurun_out/r05r; mkdir -p $o
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 3 "$o/$name.log" | cut -c1-400 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -30 "$o/$name.log" >&2; exit $rc; fi; }
step pytest 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step decmodes 600 python -u tools/decmodes.py 7,1,6 fio4k,fio4k_64k,fio4k_16k,fio4k_4k,sil4k
grep "==" $o/decmodes.log | cut -c1-300 >&2
step bench_fio4k 420 python -u bench.py --workload fio4k --no-single-call
step bench 400 python -u bench.py --no-cpu-baseline --no-e2e
