#!/bin/bash
# bench.py over every BASELINE workload (one line each).
#   tools/workloads.sh [extra bench args]
mkdir -p gpurun_out
for w in silesia64k sg512 fio4k text256k; do
  timeout -k 10 600 python -u bench.py --workload $w --steps 5 --warmup 2 --no-single-call "$@" \
      > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -20 gpurun_out/bench_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$w.json').read().splitlines()[-1]); print(d['config']['name'], 'value', d['value'], 'comp_ms', d['compress_ms'], 'dec_ms', d['decompress_ms'], 'ratio', d['ratio'], 'delta', d['ratio_delta_vs_ref'])"
done
