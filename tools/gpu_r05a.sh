#!/bin/bash
# Round 5: every -m gpu test, then the default bench (with the block floor and its clock probe).
tag=${1:-r05a}
o=gpurun_out/$tag; mkdir -p $o
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 3 "$o/$name.log" | cut -c1-1500 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi; }
step pytest 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 400 python -u bench.py
