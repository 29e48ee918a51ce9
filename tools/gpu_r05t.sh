#!/bin/bash
# Round 5: group decoder with literal + match loads fused -- decoder parity
# tests, decoders side by side, fio4k line.
o=gpurun_out/r05t; mkdir -p $o
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 3 "$o/$name.log" | cut -c1-400 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -30 "$o/$name.log" >&2; exit $rc; fi; }
step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "error_codes or small or batch_vs_oracle or group or single or every_frame or dictionary"
step decmodes 600 python -u tools/decmodes.py 7 fio4k,fio4k_64k,sil4k
step bench_fio4k 420 python -u bench.py --workload fio4k --no-single-call --no-cpu-baseline --no-e2e
