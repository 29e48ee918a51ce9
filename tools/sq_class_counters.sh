#!/bin/bash
export TMPDIR=/tmp
out=gpurun_out/sqc; mkdir -p $out
for cls in ints text records; do
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -T -d $out/${cls}1 -o run --output-format csv -- python3 tools/sq_class.py $cls 256 > $out/${cls}1.log 2>&1 || { tail -5 $out/${cls}1.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD -T -d $out/${cls}2 -o run --output-format csv -- python3 tools/sq_class.py $cls 256 > $out/${cls}2.log 2>&1 || { tail -5 $out/${cls}2.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
for cls in ("ints","text","records"):
  for p in ("1","2"):
    f=glob.glob(f"gpurun_out/sqc/{cls}{p}/run_counter_collection.csv")
    if not f: print("missing", cls, p); continue
    agg={}
    for r in csv.DictReader(open(f[0])):
        k=r['Kernel_Name'][:24]
        if 'compress' not in k: continue
        agg.setdefault(k,{}).setdefault(r['Counter_Name'],[]).append(float(r['Counter_Value']))
    for k,d in agg.items():
        print(cls, p, k, {c: round(v[-1]) for c,v in d.items()})
PY
