#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout 300 "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -n 40 gpurun_out/pytest_gpu.log
exit $rc
