#!/bin/bash
# Round 5: decode/compress overlap experiment (tools/overlap_exp.py).
tag=${1:-r05j}
o=gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 6 "$o/$name.log" | cut -c1-900 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -20 "$o/$name.log" >&2; exit $rc; fi; }
step ov_sil 300 python -u tools/overlap_exp.py silesia64k 20
step ov_t256 300 python -u tools/overlap_exp.py text256k 10
step ov_fio 300 python -u tools/overlap_exp.py fio4k 10
step ov_sg 300 python -u tools/overlap_exp.py sg512 20
