#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 120 ./exp/latency > gpurun_out/latency.log 2>&1 || exit 1
cat gpurun_out/latency.log
timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps_lds.log 2>&1 || exit 1
grep -E "^==|class " gpurun_out/stamps_lds.log | head -20
