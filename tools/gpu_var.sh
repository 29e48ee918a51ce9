#!/bin/bash
# Bench each library variant under lz4-sgori_amd/build/var (LZ4E_LIB), after
# the default build, default workload.
o=gpurun_out/var; mkdir -p $o
B=(--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-single-call --no-strong)
timeout -k 10 300 python -u bench.py "${B[@]}" > $o/default.log 2>&1 || exit $?
grep -o '"compress_ms": [0-9.]*' $o/default.log >&2
for f in lz4-sgori_amd/build/var/*.so; do
  n=$(basename $f .so)
  LZ4E_LIB=$PWD/$f timeout -k 10 300 python -u bench.py "${B[@]}" > $o/$n.log 2>&1 || exit $?
  echo "$n $(grep -o '"compress_ms": [0-9.]*\|"frames_identical": [0-9]*' $o/$n.log | tr '\n' ' ')" >&2
done
