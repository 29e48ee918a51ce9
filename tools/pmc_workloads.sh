#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, one --pmc pass each) of the
# non-default workloads, merged into a copy of profiles/pmc_traffic.json at
# gpurun_out/<tag>/pmc_traffic.json (tools/pmc_summary.py).
tag=${1:-pmcw}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
cp profiles/pmc_traffic.json $out/pmc_traffic.json
args=(--steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-single-call --no-parity --no-strong --no-decompress-only)
for w in ${WORKLOADS:-text256k fio4k sg512}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$out/$w/$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    echo "== $w $c" >&2
    timeout -s KILL 300 rocprofv3 --pmc $c -T -d $d -o run --output-format csv -- python3 bench.py --workload $w "${args[@]}" > $out/${w}_$c.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "stopping: $w $c rc=$rc" >&2; tail -5 $out/${w}_$c.log >&2; exit $rc; fi
  done
  python3 tools/pmc_summary.py $out/$w $w $out/pmc_traffic.json >&2 || exit $?
done
echo done >&2
