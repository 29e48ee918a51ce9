#!/bin/bash
# Round-4 check: every -m gpu test, then the bench lines of fio4k and the default workload.
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r04/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r04/pytest_gpu.log
timeout -k 10 300 python -u bench.py --workload fio4k > gpurun_out/r04/bench_fio4k.json 2> gpurun_out/r04/bench_fio4k.err || { tail -20 gpurun_out/r04/bench_fio4k.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench_fio4k.json').read().strip().splitlines()[-1]); print('fio4k', d['value'], d['compress_ms'], d['decompress_ms'])"
