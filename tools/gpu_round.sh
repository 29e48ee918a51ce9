#!/bin/bash
# One GPU session: smoke -> parity tests -> bench.  Stops at the first step
# that faults, aborts, times out or hangs (any exit code other than 0/1).
#   tools/gpu_round.sh [pytest -k expression]
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
K=${1:+-k "$1"}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread $K
step bench 600 python -u bench.py --steps 10 --warmup 3
