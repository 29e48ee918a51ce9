#!/bin/bash
# Chunked decoder diagnostics: stamped per-class breakdown, then the A/B of
# the decoders and of every build/var variant (tools/gpu_dec4.sh).
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ckstamps.py > gpurun_out/ckstamps.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ckstamps.txt; [ $rc -ne 0 ] && exit $rc
MODES=${MODES:-2,1,4} WL=${WL:-silesia,text256k,fio4k} bash tools/gpu_dec4.sh
