#!/bin/bash
# A/B of compress builds on the BASELINE workloads: tools/ab_compress.sh lib1.so [lib2.so ...]
# (kernel times by HIP events, tools/ktime.py; the in-tree library first)
mkdir -p gpurun_out
out=gpurun_out/ab_compress.log
: > $out
for l in "" "$@"; do
  LZ4E_LIB=$l timeout -k 10 300 python3 tools/ktime.py >> $out 2>&1 || { cat $out; exit 1; }
  LZ4E_LIB=$l timeout -k 10 120 python3 tools/single_call_trace.py 300 >> $out 2>&1 || { cat $out; exit 1; }
done
grep -v amdgpu.ids $out
