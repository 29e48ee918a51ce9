#!/bin/bash
# Streaming decoder A/B: decoder-mode GPU tests, then bench lines with the
# default decoder and with LZ4E_DECOMPRESS_MODE=s (2-wave streaming decoder).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread \
  -k "huge_runs or periodic or pipelined_vs_wave or error_codes or dict_decompress or full_size_every_frame" > gpurun_out/stream_tests.log 2>&1 || { tail -30 gpurun_out/stream_tests.log; exit 1; }
tail -3 gpurun_out/stream_tests.log
for w in ${WL:-silesia64k text256k}; do
  for m in p s; do
    LZ4E_DECOMPRESS_MODE=$m timeout -k 10 300 python -u bench.py --workload $w --steps ${BV_STEPS:-10} --warmup 3 --no-cpu-baseline --no-e2e --no-single-call --no-parity --no-strong --no-decompress-only > gpurun_out/bv.json 2>gpurun_out/bv.err || { echo "$m $w failed"; tail gpurun_out/bv.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bv.json').read().splitlines()[-1]); print('$m', '$w', d['value'], d['compress_ms'], d['decompress_ms'])"
  done
done
