#!/bin/bash
# Round 5: kernel stats + FETCH/WRITE of the default bench (batch launches
# only), then the fused round-trip experiment (tools/rtexp).
tag=${1:-r05i}
o=gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc" >&2; tail -n 6 "$o/$name.log" | cut -c1-600 >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -20 "$o/$name.log" >&2; exit $rc; fi; }
step prof 900 bash tools/profile.sh r05
cp $(find gpurun_out/prof_r05/trace -name "*kernel_stats.csv" | head -1) $o/kernel_stats.csv
python3 tools/pmc_summary.py gpurun_out/prof_r05 silesia64k $o/pmc_traffic.json > $o/pmc_summary.log 2>&1
step rt 300 python -u tools/rtexp/rtbench.py silesia64k,text256k,fio4k,sg512 20
