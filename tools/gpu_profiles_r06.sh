#!/bin/bash
# Round-6 profile refresh: rocprofv3 kernel trace + stats and the two HBM
# counter passes over the default bench (tools/profile.sh), the fio4k
# workload's counter passes (tools/pmc_workloads.sh), then the bench lines of
# the other BASELINE workloads.  Everything under gpurun_out/r06p/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r06p
bash tools/profile.sh r06 > gpurun_out/r06p/profile.log 2>&1 || { tail -20 gpurun_out/r06p/profile.log; exit 1; }
WORKLOADS=fio4k bash tools/pmc_workloads.sh r06p/pmcw > gpurun_out/r06p/pmcw.log 2>&1 || { tail -20 gpurun_out/r06p/pmcw.log; exit 1; }
for w in fio4k sg512 text256k; do
  LZ4E_CHUNK_PROF=1 timeout -k 10 400 python3 -u bench.py --workload $w --no-single-call > gpurun_out/r06p/bench_$w.json 2> gpurun_out/r06p/bench_$w.err || { tail -20 gpurun_out/r06p/bench_$w.err; exit 1; }
  tail -c 400 gpurun_out/r06p/bench_$w.json; echo
done
echo done
