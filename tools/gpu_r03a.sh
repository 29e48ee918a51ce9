#!/bin/bash
# Round-3 session A: the changed host paths (coalesced single calls, stats
# rule, watchdog reporting) and the new full-size SG-layout test, then the
# bench's single-call leg.
mkdir -p gpurun_out/r03a
o=gpurun_out/r03a
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 6 "$o/$name.log" >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "single_calls or sg512_layout or chunk or kat or edge"
step bench 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e
