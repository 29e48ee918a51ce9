#!/bin/bash
# rocprofv3 passes over the default bench: kernel trace + stats, then one
# PMC pass per HBM counter (FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Usage: tools/profile.sh <tag> [bench args...]
tag=${1:-r01}; shift
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p "$out"
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(--steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-single-call --no-parity --no-strong)
set -o pipefail
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$out/trace" -o run --output-format csv -- python3 bench.py "${args[@]}" > "$out/trace.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T -d "$out/fetch" -o run --output-format csv -- python3 bench.py "${args[@]}" > "$out/fetch.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T -d "$out/write" -o run --output-format csv -- python3 bench.py "${args[@]}" > "$out/write.log" 2>&1 || exit $?
find "$out" -name "*.csv" | head -20
