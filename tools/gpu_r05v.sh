#!/bin/bash
# Round 5 final build (group decoder, one wave per workgroup): smoke, every
# -m gpu test, decoders side by side, the fio4k and default lines.
o=gpurun_out/r05v; mkdir -p $o
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 2 "$o/$name.log" | cut -c1-300 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -30 "$o/$name.log" >&2; exit $rc; fi; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step pytest 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step decmodes 600 python -u tools/decmodes.py 7,1,6 fio4k,fio4k_16k,fio4k_4k,sil4k
step bench_fio4k 420 python -u bench.py --workload fio4k --no-single-call
step bench 500 python -u bench.py
