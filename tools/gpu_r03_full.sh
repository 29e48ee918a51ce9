#!/bin/bash
# Round-3 profile session: tools/gpu_full.sh (smoke, every -m gpu test, the
# default bench, rocprofv3 kernel trace + FETCH/WRITE passes, the other
# workloads), then the SQ instruction-mix passes.
bash tools/gpu_full.sh r03 || exit $?
bash tools/pmc_sq.sh r03/sq > gpurun_out/r03/sq_summary.log 2>&1 || { tail -5 gpurun_out/r03/sq_summary.log; exit 1; }
echo sq done >&2
