#!/bin/bash
# parity, then per-class stamps (HBM input) and a short bench
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
LZ4E_COMPRESS_LDS_MAX=0 timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || exit 1
grep -E "^==|class " gpurun_out/stamps.log | head -40
LZ4E_COMPRESS_LDS_MAX=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || exit 1
tail -n 2 gpurun_out/bench.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_lds.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_lds.log
