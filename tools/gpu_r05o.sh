#!/bin/bash
# Round 5: record slots between the pipelined decoder's parser and copiers
# (LZ4E_PIPE_RECS 4 = library, 6 / 8 / 12 = build/var): decoder parity tests
# and the decoders side by side per variant.
o=gpurun_out/r05o; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/decmodes.py 2 silesia,text256k > $o/decmodes_lib.txt 2>&1 || { cat $o/decmodes_lib.txt; exit 1; }
grep "==" $o/decmodes_lib.txt | cut -c1-200
for f in lz4-sgori_amd/build/var/lib*.so; do
  n=$(basename $f .so)
  LZ4E_LIB=$PWD/$f timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "error_codes or pipelined_vs_wave or periodic or huge or batch_vs_oracle or dictionary or every_frame" > $o/pytest_$n.log 2>&1 || { tail -30 $o/pytest_$n.log; exit 1; }
  echo "-- $n: $(tail -1 $o/pytest_$n.log)"
  LZ4E_LIB=$PWD/$f timeout -k 10 300 python -u tools/decmodes.py 2 silesia,text256k > $o/decmodes_$n.txt 2>&1 || { cat $o/decmodes_$n.txt; exit 1; }
  grep "==" $o/decmodes_$n.txt | cut -c1-200
done
timeout -k 10 300 python -u tools/decmodes.py 2 silesia > $o/decmodes_lib_again.txt 2>&1 || { cat $o/decmodes_lib_again.txt; exit 1; }
grep "==" $o/decmodes_lib_again.txt | cut -c1-200
