#!/bin/bash
# Quick A/B: compress parity tests, then the default bench twice and text256k.
tag=${1:-q}
o=gpurun_out/$tag; mkdir -p $o
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 2 "$o/$name.log" | cut -c1-900 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi; }
step pytest 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "compress or kat or edge or full_size"
B=(--steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-e2e --no-single-call --no-strong)
step bench 300 python -u bench.py "${B[@]}"
step bench2 300 python -u bench.py "${B[@]}"
step bench_t256 300 python -u bench.py --workload text256k "${B[@]}"
