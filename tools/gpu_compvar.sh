#!/bin/bash
# Compress variants A/B: each lz4-sgori_amd/build/var/lib*.so in turn as the
# library (box copy only), tools/comp_order.py kernel times.
mkdir -p gpurun_out
so=lz4-sgori_amd/lz4e_amd/liblz4e_amd.so
cp $so /tmp/orig.so
for v in lz4-sgori_amd/build/var/lib*.so; do
  cp $v $so
  echo "=== $v"
  timeout -k 10 300 python -u tools/comp_order.py > gpurun_out/compvar.txt 2>&1 || { cat gpurun_out/compvar.txt; exit 1; }
  cat gpurun_out/compvar.txt
done
cp /tmp/orig.so $so
