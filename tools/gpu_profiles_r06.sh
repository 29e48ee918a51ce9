#!/bin/bash
# Round-6 profile refresh: rocprofv3 kernel trace + stats and the two HBM
# counter passes over the default bench (tools/profile.sh), the fio4k
# workload's kernel trace, counter passes (tools/pmc_workloads.sh) and SQ
# instruction counts (tools/pmc_sq.sh), then the bench lines of the other
# BASELINE workloads.  Everything under gpurun_out/r06p/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r06p
bash tools/profile.sh r06 > gpurun_out/r06p/profile.log 2>&1 || { tail -20 gpurun_out/r06p/profile.log; exit 1; }
WORKLOADS=fio4k bash tools/pmc_workloads.sh r06p/pmcw > gpurun_out/r06p/pmcw.log 2>&1 || { tail -20 gpurun_out/r06p/pmcw.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r06p/fio_trace -o run --output-format csv -- python3 bench.py --workload fio4k --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-single-call --no-parity --no-strong > gpurun_out/r06p/fio_trace.log 2>&1 || { tail -20 gpurun_out/r06p/fio_trace.log; exit 1; }
BENCH_ARGS="--workload fio4k" bash tools/pmc_sq.sh r06p/sqfio > gpurun_out/r06p/sqfio.log 2>&1 || { tail -20 gpurun_out/r06p/sqfio.log; exit 1; }
for w in fio4k sg512 text256k; do
  LZ4E_CHUNK_PROF=1 timeout -k 10 400 python3 -u bench.py --workload $w --no-single-call > gpurun_out/r06p/bench_$w.json 2> gpurun_out/r06p/bench_$w.err || { tail -20 gpurun_out/r06p/bench_$w.err; exit 1; }
  tail -c 300 gpurun_out/r06p/bench_$w.json; echo
done
echo done
