#!/bin/bash
# Round-4 check session: smoke, every -m gpu test, the default bench, then the
# drop-in single calls under each path (round-4 A/B: direct host-mapped with the chunked /
# one-wave decoder, and the staged path).
tag=${1:-r04}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -n 4 "$out/$name.log" >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
step bench 600 python -u bench.py --steps 20 --warmup 3
sc=(--steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-parity --no-strong)
step single_direct_chunk 300 python -u bench.py "${sc[@]}"
LZ4E_DECOMPRESS_MODE=w step single_direct_wave 300 python -u bench.py "${sc[@]}"
LZ4E_NO_DIRECT=1 step single_staged 300 python -u bench.py "${sc[@]}"
echo done >&2
