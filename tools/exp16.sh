#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ktime.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || exit 1
grep -E "^==|^   " gpurun_out/stamps.log | head -40
