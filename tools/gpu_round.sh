#!/bin/bash
# One GPU session: smoke -> parity tests -> bench.  Stops at the first step
# that faults, aborts, times out or hangs (exit codes other than 0/1).
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -n 30 "gpurun_out/$name.log" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -q -rf --timeout 300
step bench 600 python bench.py --steps 3 --warmup 1
