#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/dstamps.py || exit $?
LZ4E_COMPRESS_LDS_MAX=0 timeout -k 10 300 python tools/stamps.py || exit $?
for w in silesia64k fio4k text256k; do
  LZ4E_COMPRESS_LDS_MAX=0 timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['name'], 'value', d['value'], 'comp', d['compress_ms'], d['compress_GiBps'], 'dec', d['decompress_ms'], d['decompress_GiBps'], 'ratio', d['ratio'])" || exit $?
done
