#!/bin/bash
# SQ instruction-mix / stall counters of the codec kernels over the default
# bench (one pass per counter group).  usage: tools/pmc_sq.sh [tag] [env...]
#   e.g. tools/pmc_sq.sh pipe LZ4E_DECOMPRESS_MODE=pipe
export TMPDIR=/tmp
tag=${1:-sq}; shift
for kv in "$@"; do export "$kv"; done
out=gpurun_out/$tag
mkdir -p $out
args=(--steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-single-call --no-parity --no-strong ${BENCH_ARGS:-})
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -T -d $out/p1 -o run --output-format csv -- python3 bench.py "${args[@]}" > $out/p1.log 2>&1 || { tail -20 $out/p1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -T -d $out/p2 -o run --output-format csv -- python3 bench.py "${args[@]}" > $out/p2.log 2>&1 || { tail -20 $out/p2.log; exit 1; }
python3 - "$out" <<'PY'
import csv, glob, sys
out = sys.argv[1]
for p in ("p1", "p2"):
    f = glob.glob(f"{out}/{p}/run_counter_collection.csv")
    if not f:
        print("missing", p)
        continue
    agg = {}
    for r in csv.DictReader(open(f[0])):
        k = r['Kernel_Name'].split('(')[0][-40:]
        if 'compress' not in k:
            continue
        agg.setdefault(k, {}).setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
    for k, d in agg.items():
        print(p, k, {c: round(v[-1]) for c, v in d.items()})
PY
