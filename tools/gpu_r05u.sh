#!/bin/bash
# Round 5: group decoder workgroup size variants on fio4k.
o=gpurun_out/${1:-r05u}; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/decmodes.py 7 fio4k,fio4k_16k > $o/decmodes_lib.txt 2>&1 || { cat $o/decmodes_lib.txt; exit 1; }
grep "==" $o/decmodes_lib.txt | cut -c1-200
for f in lz4-sgori_amd/build/var/lib*.so; do
  n=$(basename $f .so)
  LZ4E_LIB=$PWD/$f timeout -k 10 300 python -u tools/decmodes.py 7 fio4k,fio4k_16k > $o/decmodes_$n.txt 2>&1 || { cat $o/decmodes_$n.txt; exit 1; }
  echo "-- $n"; grep "==" $o/decmodes_$n.txt | cut -c1-200
done
timeout -k 10 300 python -u tools/decmodes.py 7 fio4k > $o/decmodes_lib_again.txt 2>&1 || { cat $o/decmodes_lib_again.txt; exit 1; }
grep "==" $o/decmodes_lib_again.txt | cut -c1-200
