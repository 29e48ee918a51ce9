#!/bin/bash
export LZ4E_COMPRESS_LDS_MAX=0
LZ4E_COMPRESS_GTABLE=1 timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout 300 -k "compress or kat or full_size" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for g in 0 1; do
  LZ4E_COMPRESS_GTABLE=$g timeout -k 10 300 python tools/stamps.py 2>&1 | grep -v "^   [a-z]* *[0-9]* *(" || exit $?
  LZ4E_COMPRESS_GTABLE=$g timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gtable=$g', d['config']['name'], 'value', d['value'], 'comp', d['compress_ms'], d['compress_GiBps'], 'dec', d['decompress_ms'], d['decompress_GiBps'])" || exit $?
done
