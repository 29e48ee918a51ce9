#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 25 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
LZ4E_COMPRESS_LDS_MAX=0 timeout -k 10 300 python tools/ktime.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python tools/ktime.py 2>&1 | grep -v amdgpu.ids
LZ4E_COMPRESS_LDS_MAX=0 timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || exit 1
grep -E "^==|class " gpurun_out/stamps.log | head -40
