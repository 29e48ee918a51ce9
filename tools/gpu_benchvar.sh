#!/bin/bash
# Library variants A/B on bench lines: each lz4-sgori_amd/build/var/lib*.so
# in turn (box copy only), silesia64k and text256k quick bench lines.
mkdir -p gpurun_out
so=lz4-sgori_amd/lz4e_amd/liblz4e_amd.so
cp $so /tmp/orig.so
for v in lz4-sgori_amd/build/var/lib*.so; do
  cp $v $so
  for w in silesia64k text256k; do
    timeout -k 10 300 python -u bench.py --workload $w --steps ${BV_STEPS:-5} --warmup 2 --no-cpu-baseline --no-e2e --no-single-call --no-parity --no-strong > gpurun_out/bv.json 2>/dev/null || { echo "$v $w failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bv.json').read().splitlines()[-1]); print('$v', '$w', d['value'], d['compress_ms'], d['decompress_ms'])"
  done
done
cp /tmp/orig.so $so
