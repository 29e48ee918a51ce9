#!/bin/bash
# Round 5: band compressor phase stamps + kernel trace.
tag=${1:-r05c}
o=gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 12 "$o/$name.log" | cut -c1-600 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi; }
step stamps 300 python -u tools/bandstamps.py silesia
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o band -- python -u tools/bandstamps.py silesia 1024
find $o/prof -name "*kernel_stats.csv" -exec cp {} $o/kernel_stats.csv \;
head -8 $o/kernel_stats.csv >&2
B=(--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-single-call --no-strong --no-parity)
step bench_band 300 python -u bench.py "${B[@]}"
