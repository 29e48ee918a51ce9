#!/bin/bash
# Round 5: decoder window with one register segment, loaded every batch --
# every -m gpu test, the silesia64k and text256k lines, decoders side by side.
tag=${1:-r05n}
o=gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 3 "$o/$name.log" | cut -c1-1200 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -30 "$o/$name.log" >&2; exit $rc; fi; }
step pytest 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 400 python -u bench.py --no-single-call --no-cpu-baseline --no-e2e
step bench_t256 400 python -u bench.py --workload text256k --no-single-call --no-cpu-baseline --no-e2e
step decmodes 600 python -u tools/decmodes.py 2,1,6,7 silesia,text256k,fio4k,sil4k
