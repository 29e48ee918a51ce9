#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "decompress or full_size or chunk or dict or periodic or pipelined" > gpurun_out/pytest_dec.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_dec.log
[ $rc -ne 0 ] && exit $rc
echo "--- ordered"; DECAB_ORDER=1 timeout -k 10 300 python -u tools/decab.py 256 > gpurun_out/decab.txt 2>&1 || { tail gpurun_out/decab.txt; exit 1; }
grep "==" gpurun_out/decab.txt | grep -E "sil|text256k"
echo "--- block order"; LZ4E_DECOMPRESS_ORDER=0 DECAB_ORDER=1 timeout -k 10 300 python -u tools/decab.py 256 > gpurun_out/decab0.txt 2>&1 || { tail gpurun_out/decab0.txt; exit 1; }
grep "==" gpurun_out/decab0.txt | grep -E "sil|text256k"
