#!/bin/bash
# Compress round: phase stamps (tools/stamps.py), the compress parity tests,
# kernel times by launch order (tools/comp_order.py), then a short bench line.
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stamps.py > gpurun_out/stamps.txt 2>&1; rc=$?
grep -E "==|setup|tables|chainwalk|slowest" gpurun_out/stamps.txt | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "compress or kat or edge or full_size or smoke" > gpurun_out/pytest_comp.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_comp.log
[ $rc -ne 0 ] && exit $rc
echo "--- launch order"; timeout -k 10 300 python -u tools/comp_order.py || exit 1
echo "--- block order"; LZ4E_COMPRESS_ORDER=0 timeout -k 10 300 python -u tools/comp_order.py || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-single-call > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err; rc=$?
python3 -c "import json; d=json.loads(open('gpurun_out/bench_quick.json').read().splitlines()[-1]); print('value', d['value'], 'comp_ms', d['compress_ms'], 'dec_ms', d['decompress_ms'], 'identical', d['parity']['frames_identical'])" || tail -5 gpurun_out/bench_quick.err
exit $rc
