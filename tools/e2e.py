"""Diagnostic: bench.py's end-to-end leg alone (lz4e_chunk_write_batch over
host bio_vec lists, PCIe-inclusive) per workload, for A/B of the chunk
pipeline's host side (LZ4E_LIB picks the library; LZ4E_CHUNK_PROF=1 adds
the per-phase host times on stderr).

usage: python tools/e2e.py [workloads, e.g. silesia64k,text256k,fio4k]"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["silesia64k", "text256k", "fio4k"]
for w in names:
    bs, cls, gen, seg, desc = bench.WORKLOADS[w]
    nblk = bench.DEFAULT_BLOCKS[w]
    U = min(nblk * bs, bench.TOTAL_BYTES.get(w, nblk * bs))
    lens = np.full(nblk, bs, dtype=np.int64)
    lens[-1] = U - (nblk - 1) * bs
    host = np.zeros(nblk * bs, np.uint8)
    host[:U] = bench.make_data(gen, U, bench.CORPUS_SEED)
    r = bench.end_to_end(host, lens, bs, seg, reps=5)
    print(json.dumps({"workload": w, "lib": os.environ.get("LZ4E_LIB", ""), **r}), flush=True)
