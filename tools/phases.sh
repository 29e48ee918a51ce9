#!/bin/bash
# Per-phase cycle breakdowns from the stamped diagnostic kernels
# (tools/stamps.py: compress, tools/dstamps.py: one-wave decoder).
mkdir -p gpurun_out
timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || exit 1
grep -E "^==|^   " gpurun_out/stamps.log | head -40
timeout -k 10 300 python tools/dstamps.py > gpurun_out/dstamps.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/dstamps.log | head -40
