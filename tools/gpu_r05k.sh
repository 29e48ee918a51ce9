#!/bin/bash
# Round 5: overlap experiment without the stream-ordered scratch allocations
# (launch order off), to see whether the pool serialises the two streams.
tag=${1:-r05k}
o=gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 6 "$o/$name.log" | cut -c1-900 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -20 "$o/$name.log" >&2; exit $rc; fi; }
LZ4E_DECOMPRESS_ORDER=0 step ov_dec0 300 python -u tools/overlap_exp.py silesia64k 20
LZ4E_DECOMPRESS_ORDER=0 LZ4E_COMPRESS_ORDER=0 step ov_both0 300 python -u tools/overlap_exp.py silesia64k 20
