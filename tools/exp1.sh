#!/bin/bash
mkdir -p gpurun_out
for w in silesia64k fio4k; do
  for lds in 65536 0; do
    echo "== $w lds_max=$lds"
    LZ4E_COMPRESS_LDS_MAX=$lds timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline || exit $?
  done
done
