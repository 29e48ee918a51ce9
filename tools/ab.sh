#!/bin/bash
# A/B kernel timings of several builds: tools/ab.sh lib1.so lib2.so ...
mkdir -p gpurun_out
export LZ4E_COMPRESS_LDS_MAX=${LZ4E_COMPRESS_LDS_MAX:-0}
timeout -k 10 300 python tools/ktime.py > gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
for l in "$@"; do
  LZ4E_LIB=$l timeout -k 10 300 python tools/ktime.py >> gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
done
cat gpurun_out/ab.log | grep -v amdgpu.ids
