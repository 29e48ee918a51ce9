#!/bin/bash
# Decoder A/B: the default library's decoders (modes $MODES, default 2,1,4)
# on $WL, then every lz4-sgori_amd/build/var/lib*.so's chunked decoder.
mkdir -p gpurun_out
WL=${WL:-classes,silesia,text256k,fio4k}
timeout -k 10 400 python -u tools/decmodes.py ${MODES:-2,1,4} $WL > gpurun_out/decmodes.txt 2>&1 || { cat gpurun_out/decmodes.txt; exit 1; }
grep "==\|!!" gpurun_out/decmodes.txt
for f in lz4-sgori_amd/build/var/lib*.so; do
  [ -e "$f" ] || continue
  n=$(basename $f .so)
  LZ4E_LIB=$PWD/$f timeout -k 10 300 python -u tools/decmodes.py 4 ${VWL:-silesia,text256k,fio4k} > gpurun_out/decmodes_$n.txt 2>&1 || { cat gpurun_out/decmodes_$n.txt; exit 1; }
  echo "-- $n"; grep "==\|!!" gpurun_out/decmodes_$n.txt
done
