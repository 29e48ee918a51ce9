#!/bin/bash
# Round 5: SQ counters of the fio4k launches (is fio4k compress issue-bound?)
export TMPDIR=/tmp
BENCH_ARGS="--workload fio4k --no-decompress-only" timeout -k 10 700 bash tools/pmc_sq.sh r05l/sqfio
