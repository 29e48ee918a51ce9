#!/bin/bash
# Streaming decoder variants: tools/streamab.py with each
# lz4-sgori_amd/build/var/lib*.so swapped in (box copy only).
mkdir -p gpurun_out
so=lz4-sgori_amd/lz4e_amd/liblz4e_amd.so
cp $so /tmp/orig.so
for v in lz4-sgori_amd/build/var/lib*.so; do
  cp $v $so
  echo "## $v"
  timeout -k 10 300 python -u tools/streamab.py ${SV_NB:-256} ${SV_KINDS:-text,ints,records} 2>&1 | grep -v amdgpu.ids
done
cp /tmp/orig.so $so
