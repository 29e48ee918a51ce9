#!/bin/bash
# Library variants A/B on single-class batches (tools/comp_class.py), then the
# GPU parity tests with the last variant installed (box copy only).
mkdir -p gpurun_out
so=lz4-sgori_amd/lz4e_amd/liblz4e_amd.so
for v in lz4-sgori_amd/build/var/lib*.so; do
  cp $v $so
  for k in ${CLASSES:-random jpeg silesia}; do
    echo -n "$v " ; timeout -k 10 300 python -u tools/comp_class.py $k 2>/dev/null || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_var.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_var.log; exit $rc
