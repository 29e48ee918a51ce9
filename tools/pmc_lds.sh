#!/bin/bash
# LDS pressure counters of the codec kernels over the default bench workload.
export TMPDIR=/tmp
out=gpurun_out/lds
mkdir -p $out
args=(--steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-single-call --no-parity --no-strong)
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS -T -d $out/p1 -o run --output-format csv -- python3 bench.py "${args[@]}" > $out/p1.log 2>&1 || { tail -20 $out/p1.log; exit 1; }
python3 - "$out" <<'PY'
import csv, glob, sys
out = sys.argv[1]
f = glob.glob(f"{out}/p1/run_counter_collection.csv")
agg = {}
for r in csv.DictReader(open(f[0])):
    k = r['Kernel_Name'].split('(')[0][-40:]
    if 'compress' not in k:
        continue
    agg.setdefault(k, {}).setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
for k, d in agg.items():
    print(k, {c: round(v[-1]) for c, v in d.items()})
PY
