#!/bin/bash
# SQ instruction-mix counters per Silesia-proxy class (256 x 64 KiB blocks
# each, tools/sq_class.py), the round-1 profile's layout.
export TMPDIR=/tmp
out=gpurun_out/sq_class
mkdir -p $out
for k in ints text records; do
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -T -d $out/$k/p1 -o run --output-format csv -- python3 tools/sq_class.py $k > $out/$k.p1.log 2>&1 || { tail $out/$k.p1.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -T -d $out/$k/p2 -o run --output-format csv -- python3 tools/sq_class.py $k > $out/$k.p2.log 2>&1 || { tail $out/$k.p2.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
for k in ("ints", "text", "records"):
    for p in ("p1", "p2"):
        f = glob.glob(f"gpurun_out/sq_class/{k}/{p}/run_counter_collection.csv")[0]
        agg = {}
        for r in csv.DictReader(open(f)):
            kn = r['Kernel_Name'].split('(')[0][-40:]
            if 'compress' not in kn or 'weight' in kn:
                continue
            agg.setdefault(kn, {}).setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
        for kn, d in agg.items():
            print(k, p, kn, {c: round(v[-1]) for c, v in d.items()})
PY
