#!/bin/bash
# Round 5: 16-lane group decoder (mode 8) -- decoder parity tests, decoders
# side by side on the small-block workloads, fio4k line with each.
o=gpurun_out/r05p; mkdir -p $o
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 3 "$o/$name.log" | cut -c1-700 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -30 "$o/$name.log" >&2; exit $rc; fi; }
step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "error_codes or small or batch_vs_oracle or lane or single"
step decmodes 600 python -u tools/decmodes.py 7,8,1 fio4k,sil4k
step bench_fio_lane 420 python -u bench.py --workload fio4k --no-single-call --no-cpu-baseline --no-e2e
LZ4E_DECOMPRESS_MODE=g step bench_fio_group 420 python -u bench.py --workload fio4k --no-single-call --no-cpu-baseline --no-e2e
