#!/bin/bash
# Round 5: band experiment -- instruction-cache / band-width question: stamps
# of the three builds on 1024 silesia-proxy blocks.
tag=${1:-r05g}
o=gpurun_out/$tag; mkdir -p $o
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; grep -E "stamped band|cycles per chain|chain split|text  |records|text block" "$o/$name.log" | cut -c1-400 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi; }
BAND_LIB=tools/bandexp/libband.so step all3 300 python -u tools/bandexp/bandstamps.py silesia 1024
BAND_LIB=tools/bandexp/libband_u16.so step u16 300 python -u tools/bandexp/bandstamps.py silesia 1024
BAND_LIB=tools/bandexp/libband512_u16.so step b512 300 python -u tools/bandexp/bandstamps.py silesia 1024
