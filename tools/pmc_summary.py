"""Per-kernel HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
(tools/profile.sh) -> bytes per launch, written to profiles/pmc_traffic.json
for bench.py's roofline.traffic.

FETCH_SIZE / WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md (HBM section) gfx950
FETCH_SIZE tallies 128-B memory requests at 64 B, i.e. reports half the bytes of
wide streaming reads: the read side is doubled (the guide calls other access
widths uncalibrated; the raw values are kept alongside).

usage: python tools/pmc_summary.py <prof dir> <workload> [out json]"""
import csv
import json
import os
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    prof, workload = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    fetch = per_kernel(os.path.join(prof, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(prof, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    res = json.load(open(out)) if os.path.exists(out) else {}
    ent = {}
    for k, d in (("compress_kernel", "compress"), ("decompress_pipe_kernel", "decompress"),
                 ("decompress_group_kernel", "decompress"), ("decompress_kernel", "decompress")):
        name = next((n for n in fetch if n.startswith(k)), None)
        if name is None or d in ent:
            continue
        f_raw = fetch[name] * 1024
        w = write.get(name, 0.0) * 1024
        ent[d] = round(2 * f_raw + w)
        ent[d + "_detail"] = {"kernel": k, "fetch_bytes_raw": round(f_raw),
                              "fetch_bytes_x2": round(2 * f_raw), "write_bytes": round(w)}
    ent["source"] = prof
    res[workload] = ent
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(ent, indent=1))


if __name__ == "__main__":
    main()
