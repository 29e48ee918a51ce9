#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || exit 1
grep -E "^==|^   " gpurun_out/stamps.log | head -40
