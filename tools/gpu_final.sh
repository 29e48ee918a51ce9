#!/bin/bash
# Round-end check on the final build: smoke, every -m gpu test, the default bench.
mkdir -p gpurun_out/final
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
timeout -k 10 600 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/final/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['compress_ms'], d['decompress_ms'], d['strong']['block_floor']['floor_ms'], d['single_call']['threads']['1'])"
