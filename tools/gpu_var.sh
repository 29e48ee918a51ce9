#!/bin/bash
# Bench each library variant under lz4-sgori_amd/build/var (LZ4E_LIB) after
# the default build, on each workload of $WORKLOADS (default silesia64k);
# prints compress / decompress ms and the parity count per run.
o=gpurun_out/var; mkdir -p $o
B=(--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-single-call --no-strong)
pick() { grep -o '"compress_ms": [0-9.]*\|"decompress_ms": [0-9.]*\|"frames_identical": [0-9]*' "$1" | tr '\n' ' '; }
for w in ${WORKLOADS:-silesia64k}; do
  timeout -k 10 300 python -u bench.py --workload $w "${B[@]}" > $o/default_$w.log 2>&1 || exit $?
  echo "$w default $(pick $o/default_$w.log)" >&2
  for f in lz4-sgori_amd/build/var/*.so; do
    n=$(basename $f .so)
    LZ4E_LIB=$PWD/$f timeout -k 10 300 python -u bench.py --workload $w "${B[@]}" > $o/${n}_$w.log 2>&1 || exit $?
    echo "$w $n $(pick $o/${n}_$w.log)" >&2
  done
done
