#!/bin/bash
# Decoder session: the decoder parity tests, then the decoders side by side
# (modes $MODES) on $WL.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "${TK:-small or error_codes or pipelined_vs_wave or periodic or huge or single_calls or batch_vs_oracle}" > gpurun_out/pytest_dec.log 2>&1 \
  || { tail -40 gpurun_out/pytest_dec.log; exit 1; }
tail -2 gpurun_out/pytest_dec.log
timeout -k 10 400 python -u tools/decmodes.py ${MODES:-2,5,1,6} ${WL:-silesia,text256k,fio4k} > gpurun_out/decmodes.txt 2>&1 \
  || { cat gpurun_out/decmodes.txt; exit 1; }
grep "==\|!!" gpurun_out/decmodes.txt
# variants (tools/build_decvar.sh): the same modes
for f in lz4-sgori_amd/build/var/lib*.so; do
  [ -e "$f" ] || continue
  n=$(basename $f .so)
  LZ4E_LIB=$PWD/$f timeout -k 10 400 python -u tools/decmodes.py ${MODES:-2,5,1,6} ${WL:-silesia,text256k,fio4k} > gpurun_out/decmodes_$n.txt 2>&1 || { cat gpurun_out/decmodes_$n.txt; exit 1; }
  echo "-- $n"; grep "==\|!!" gpurun_out/decmodes_$n.txt
done
