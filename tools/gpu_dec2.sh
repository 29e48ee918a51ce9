#!/bin/bash
# Decoder A/B session: decoder parity tests, then the default bench with the
# sequence-level copy stage (copy_fast2) and the byte-pointer one
# (LZ4E_DEC_COPY=1), then the per-class phase counters of both.
mkdir -p gpurun_out/dec2
o=gpurun_out/dec2
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 5 "$o/$name.log" >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi; }
step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "decompress or periodic or full_size or chunk or smoke or dict"
B=(--steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-e2e --no-single-call --no-strong)
step bench_c2 300 python -u bench.py "${B[@]}"
LZ4E_DEC_COPY=1 step bench_c1 300 python -u bench.py "${B[@]}"
step bench_c2b 300 python -u bench.py "${B[@]}"
step bench_t256_c2 300 python -u bench.py --workload text256k "${B[@]}"
LZ4E_DEC_COPY=1 step bench_t256_c1 300 python -u bench.py --workload text256k "${B[@]}"
step decab_c2 300 python -u tools/decab.py 256
