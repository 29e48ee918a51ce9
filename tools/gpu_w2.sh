#!/bin/bash
# 128-position-window compressor A/B (LZ4E_COMPRESS_W2=1, lz4e_window2.h):
# the compress parity tests with the switch on, then the bench with and
# without it on three workloads, and the W2 per-phase stamps.
tag=${1:-w2}
o=gpurun_out/$tag; mkdir -p $o
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 3 "$o/$name.log" >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi; }
B=(--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-single-call --no-strong)
export LZ4E_COMPRESS_W2=1
step pytest_w2 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "compress or kat or edge or full_size or sg"
step bench_w2 300 python -u bench.py "${B[@]}"
step bench_t256_w2 300 python -u bench.py --workload text256k "${B[@]}"
step bench_fio_w2 300 python -u bench.py --workload fio4k "${B[@]}"
step stamps_w2 300 python -u tools/stamps.py
export LZ4E_COMPRESS_W2=0
step bench_w1 300 python -u bench.py "${B[@]}"
step bench_t256_w1 300 python -u bench.py --workload text256k "${B[@]}"
step bench_fio_w1 300 python -u bench.py --workload fio4k "${B[@]}"
for f in $o/bench*.log; do echo "$(basename $f) $(grep -o '"compress_ms": [0-9.]*\|"frames_identical": [0-9a-z]*\|"value": [0-9.]*' $f | tr '\n' ' ')" >&2; done
