#!/bin/bash
# Kernel + memory-copy trace of the drop-in single calls (tools/single_call_trace.py).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/single_call_trace.py 300 > gpurun_out/single_plain.log 2>&1 || { tail gpurun_out/single_plain.log; exit 1; }
cat gpurun_out/single_plain.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/profsingle -o run -- python3 tools/single_call_trace.py 300 > gpurun_out/profsingle.log 2>&1 || { tail -20 gpurun_out/profsingle.log; exit 1; }
grep "single" gpurun_out/profsingle.log
python3 tools/rocpd_stats.py $(find gpurun_out/profsingle -name "*.db" | head -1) | head -12
