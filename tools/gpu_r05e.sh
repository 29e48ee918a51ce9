#!/bin/bash
# Round 5: band compressor phase stamps (chain split) on silesia 1024 blocks.
tag=${1:-r05e}
o=gpurun_out/$tag; mkdir -p $o
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 14 "$o/$name.log" | cut -c1-600 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi; }
step stamps 300 python -u tools/bandstamps.py silesia 1024
