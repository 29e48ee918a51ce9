#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for lds in 65536 0; do
  LZ4E_COMPRESS_LDS_MAX=$lds timeout -k 10 300 python tools/stamps.py || exit $?
  LZ4E_COMPRESS_LDS_MAX=$lds timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit $?
done
