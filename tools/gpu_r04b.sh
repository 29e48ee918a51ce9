#!/bin/bash
# Round-4 profile session: rocprofv3 kernel trace + FETCH / WRITE passes of
# the default bench, the SQ instruction-mix passes, the other BASELINE
# workloads, and the decoder A/B (tools/decmodes.py).
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
step bench 600 python -u bench.py
cp $out/bench.log $out/bench.json
args=(--steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-single-call --no-parity --no-strong)
step prof_trace 300 rocprofv3 --kernel-trace --stats -T -d $out/trace -o run --output-format csv -- python3 bench.py "${args[@]}"
cp $(find $out/trace -name "*kernel_stats.csv" | head -1) $out/kernel_stats.csv 2>/dev/null
step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE -T -d $out/fetch -o run --output-format csv -- python3 bench.py "${args[@]}"
step prof_write 300 rocprofv3 --pmc WRITE_SIZE -T -d $out/write -o run --output-format csv -- python3 bench.py "${args[@]}"
python3 tools/pmc_summary.py $out silesia64k $out/pmc_traffic.json > $out/pmc_summary.log 2>&1
step sq 700 bash tools/pmc_sq.sh $tag/sq
for w in fio4k sg512 text256k; do
  step bench_$w 600 python -u bench.py --workload $w --steps 5 --warmup 2 --no-single-call
done
LZ4E_COMPRESS_LDS_MAX=0 step bench_fio4k_hbm_input 600 python -u bench.py --workload fio4k --steps 5 --warmup 2 --no-single-call --no-e2e --no-cpu-baseline --no-strong
step decmodes 600 python -u tools/decmodes.py 2,1,6,7,5,4 silesia,text256k,fio4k,sil4k
step wavestamps 300 python -u tools/wavestamps.py 1,6,7 fio4k,sil4k
step single_call_modes 300 bash -c 'for m in s w l; do LZ4E_DECOMPRESS_MODE=$m python3 tools/single_call_trace.py 300 | sed "s/^/$m: /"; done'
step prof_single 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $out/profsingle -o run -- python3 tools/single_call_trace.py 300
python3 tools/rocpd_stats.py $(find $out/profsingle -name "*.db" | head -1) > $out/single_call_kernels.txt 2>&1
echo done >&2
