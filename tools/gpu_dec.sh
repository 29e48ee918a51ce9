#!/bin/bash
# Decoder round: parity tests of both decoders, then the A/B kernel times.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "decompress or full_size or chunk or dict or periodic or pipelined" > gpurun_out/pytest_dec.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_dec.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/decab.py ${1:-256} > gpurun_out/decab.txt 2>&1; rc=$?; grep -A1 "==" gpurun_out/decab.txt; exit $rc
