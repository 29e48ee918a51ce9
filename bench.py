#!/usr/bin/env python3
"""bench.py -- LZ4E scatter-gather block codec on MI355X (BASELINE.json metric).

Metric: GiB/s compress+decompress (round trip, whole job), 64 KiB blocks,
plus the ratio delta vs the reference (0 by construction: frames are
bit-identical, checked on a sample against the CPU oracle every run).

A step = one pass of the hot path over one batch of synthetic input already
resident in HBM: LZ4E compress of every block (one launch), then LZ4E safe
decompress of every frame (one launch).  value = uncompressed bytes of all
ranks / max-over-ranks step time.

Default workload (configs[1] of BASELINE.json): Silesia-proxy, 3234 blocks of
64 KiB (~212 MB, the Silesia corpus size) per GPU, each block a 16 x 4 KiB
bio_vec list (byU16 hash table).  Other workloads (--workload) are the parity
configurations: fio4k (configs[2]), sg512 (configs[3], byU32), text256k
(configs[4], decompress-only reported separately).

Multi-GPU (torch.distributed.run, one rank per GPU): blocks are independent,
each rank owns its own shard (weak scaling, no data-path collective); the
only collectives (lz4e_amd.shards) are the frame-stream layout all_gather and
the max-over-ranks reduction of the timing.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))

import lz4e_amd  # noqa: E402
from lz4e_amd import BYU16, BYU32, corpus  # noqa: E402
from lz4e_amd.shards import frame_layout, reduce_step  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

WORKLOADS = {
    # name: (block bytes, table class, generator, description)
    "silesia64k": (65536, BYU16, "silesia",
                   "Silesia-proxy, 64 KiB independent blocks (16 x 4 KiB bio_vecs, byU16), round trip"),
    "fio4k": (4096, BYU16, "fio",
              "fio buffer_compress_percentage=50 pattern, 4 KiB chunks (1 x 4 KiB bio_vec, byU16), round trip"),
    "sg512": (65536, BYU32, "silesia",
              "Silesia-proxy, 64 KiB blocks of 128 x 512 B bio_vecs (byU32), round trip"),
    "text256k": (262144, BYU32, "text",
                 "enwik9-proxy text, 256 KiB blocks (1 bio_vec, byU32), round trip"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="silesia64k", choices=sorted(WORKLOADS))
    ap.add_argument("--blocks", type=int, default=0, help="blocks per GPU (0: workload default)")
    ap.add_argument("--cpu-blocks", type=int, default=0, help="CPU baseline sample size in blocks")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive chunk-layer run")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def make_data(gen: str, nbytes: int, seed: int) -> np.ndarray:
    if gen == "silesia":
        return corpus.silesia_proxy(nbytes, seed)
    if gen == "fio":
        return corpus.fio_pattern(nbytes, seed)
    return corpus.text_proxy(nbytes, seed)


def end_to_end(host: np.ndarray, nblk: int, bs: int, cls: int, reps: int = 3) -> dict:
    """lz4e_chunk_write_batch over the same blocks given as host bio_vec lists
    (16 x 4 KiB segments per 64 KiB block, 128 x 512 B for sg512): SG gather
    -> H2D -> compress -> decompress -> D2H -> copy-out, four pipeline slots.
    The host buffers are pageable numpy memory, as a bio's pages would be."""
    import ctypes
    seg = 512 if cls == BYU32 and bs == 65536 else min(bs, 4096)
    nseg = bs // seg
    base = host.ctypes.data
    bv = (lz4e_amd.BioVec * (nblk * nseg))()
    addr = np.frombuffer(bv, dtype=np.dtype([("p", "<u8"), ("l", "<u4"), ("o", "<u4")]))
    addr["p"] = base + np.arange(nblk * nseg, dtype=np.uint64) * seg
    addr["l"] = seg
    addr["o"] = 0
    its = (lz4e_amd.BvecIter * nblk)()
    out = np.empty(nblk * bs, np.uint8)
    reqs = (lz4e_amd.ChunkRequest * nblk)()
    bvp = ctypes.cast(bv, ctypes.c_void_p).value
    for i in range(nblk):
        its[i].bi_size = bs
        reqs[i].src = ctypes.cast(bvp + i * nseg * ctypes.sizeof(lz4e_amd.BioVec),
                                  ctypes.POINTER(lz4e_amd.BioVec))
        reqs[i].srcIter = ctypes.pointer(its[i])
        reqs[i].data = out.ctypes.data + i * bs
    L = lz4e_amd.lib()
    times = []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        good = L.lz4e_chunk_write_batch(reqs, nblk, None)
        times.append(time.perf_counter() - t0)
        if good != nblk:
            raise SystemExit(f"bench: chunk pipeline failed ({good}/{nblk}): {lz4e_amd.last_error()}")
    if not np.array_equal(out, host[:nblk * bs]):
        raise SystemExit("bench: chunk pipeline round trip mismatch")
    t = float(np.median(times[1:]))
    return {"value": round(nblk * bs / t / 2**30, 3), "unit": "GiB/s", "ms": round(t * 1e3, 2),
            "path": f"lz4e_chunk_write_batch: {nblk} WRITE bios of {nseg} x {seg} B host segments, "
                    "SG gather -> H2D -> compress -> decompress -> D2H -> copy-out (PCIe-inclusive)"}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)
    if not lz4e_amd.gpu_available():
        raise SystemExit("bench: HIP path unavailable: " + lz4e_amd.last_error())

    bs, cls, gen, desc = WORKLOADS[args.workload]
    default_blocks = {65536: 3234, 4096: 262144 // 4, 262144: 3815 // 4}[bs]
    nblk = args.blocks or default_blocks
    U = nblk * bs
    host = make_data(gen, U, 0x5157 + 7919 * rank)

    # ---- device-resident layout ------------------------------------------
    offs = np.arange(nblk, dtype=np.int64) * bs
    lens = np.full(nblk, bs, dtype=np.int32)
    cap1 = bs + bs // 255 + 16
    caps = np.full(nblk, cap1, dtype=np.int32)
    slot = (cap1 + 64 + 15) // 16 * 16
    doffs = np.arange(nblk, dtype=np.int64) * slot
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).to(dev)
    d_src = torch.from_numpy(host).to(dev)
    d_off, d_len, d_tt = t(offs, np.int64), t(lens, np.int32), t(np.full(nblk, cls), np.uint8)
    d_dst = torch.zeros(nblk * slot, dtype=torch.uint8, device=dev)
    d_doff, d_cap = t(doffs, np.int64), t(caps, np.int32)
    d_ret = torch.zeros(nblk, dtype=torch.int32, device=dev)
    d_out = torch.zeros(U + 64, dtype=torch.uint8, device=dev)
    d_dret = torch.zeros(nblk, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def compress():
        lz4e_amd.compress_batch_dev(d_src, d_off, d_len, d_tt, d_dst, d_doff, d_cap, d_ret,
                                    max_len=bs, stream=stream.cuda_stream)

    def decompress():
        lz4e_amd.decompress_batch_dev(d_dst, d_doff, d_ret, d_out, d_off, d_len, d_dret,
                                      stream=stream.cuda_stream)

    for _ in range(max(1, args.warmup)):
        compress()
        decompress()
    torch.cuda.synchronize(dev)

    # ---- correctness gate (every run) ---------------------------------------
    rets = d_ret.cpu().numpy()
    if (rets <= 0).any() or not torch.equal(d_out[:U], d_src) or not (d_dret == bs).all():
        raise SystemExit("bench: round trip mismatch")
    C = int(rets.astype(np.int64).sum())
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ref  # checker only: sample frames must equal the oracle's

    dst_host = d_dst.cpu().numpy()
    sample = list(range(0, nblk, max(1, nblk // 16)))[:16]
    for i in sample:
        er, ef, _, _ = oracle_ref.compress(host[offs[i]:offs[i] + bs].tobytes(), cls)
        got = dst_host[doffs[i]:doffs[i] + rets[i]].tobytes()
        if er != rets[i] or got != ef:
            raise SystemExit(f"bench: frame {i} differs from the oracle")

    # ---- timed region ----------------------------------------------------------
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for e0, e1, e2 in ev:
        e0.record(stream)
        compress()
        e1.record(stream)
        decompress()
        e2.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    comp_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))
    dec_ms = float(np.mean([b.elapsed_time(c) for _, b, c in ev]))
    step_s = elapsed / args.steps
    group = dist.group.WORLD if dist else None
    # this rank's place in the job's frame stream (all_gather + exclusive scan)
    _, C_all, _ = frame_layout(C, nblk, group, dev)
    (step_s, comp_ms, dec_ms), _ = reduce_step([step_s, comp_ms, dec_ms], C, group, dev)
    U_all = U * world
    value = U_all / step_s / 2**30

    # ---- roofline of the dominant kernel ---------------------------------------
    dom = "compress" if comp_ms >= dec_ms else "decompress"
    dom_ms = max(comp_ms, dec_ms)
    achieved = (U + C) / (dom_ms / 1e3) / 1e9  # algorithmic U + C bytes per launch
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            traffic = tj.get(args.workload, {}).get(dom)
        except Exception:
            traffic = None
    roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "algorithmic_bytes_per_launch": int(U + C)}

    result = {
        "metric": "GiB/s compress+decompress (whole node), 64 KiB blocks; ratio delta vs ref",
        "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": desc, "name": args.workload, "blocks_per_gpu": nblk,
                   "block_bytes": bs, "table_type": {1: "byU16", 3: "byU32", 7: "byU64"}[cls],
                   "bytes_per_gpu": U, "parallelism": f"dp{world} (block shards)"},
        "ratio": round(U_all / C_all, 5), "ratio_delta_vs_ref": 0.0,
        "compress_ms": round(comp_ms, 4), "decompress_ms": round(dec_ms, 4),
        "compress_GiBps": round(U_all / (comp_ms / 1e3) / 2**30, 3),
        "decompress_GiBps": round(U_all / (dec_ms / 1e3) / 2**30, 3),
        "roofline": roofline,
    }

    # ---- end to end through the chunk layer (PCIe-inclusive, never `value`) ----
    if world == 1 and not args.no_e2e:
        result["end_to_end"] = end_to_end(host, nblk, bs, cls)

    # ---- CPU baseline (rank 0, N=1 only) ---------------------------------------
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or max(1, min(16, os.cpu_count() or 1))
        nb = args.cpu_blocks or min(nblk, max(threads * 4, (64 << 20) // bs))
        L = oracle_ref.load()
        c_off = np.ascontiguousarray(offs[:nb].astype(np.uint64))
        c_len = np.ascontiguousarray(lens[:nb].astype(np.uint32))
        c_tt = np.full(nb, cls, np.uint8)
        c_cap = np.full(nb, cap1, np.uint32)
        c_doff = np.ascontiguousarray(doffs[:nb].astype(np.uint64))
        c_out = np.zeros(nb * slot, np.uint8)
        c_ret = np.zeros(nb, np.int32)
        c_dec = np.zeros(nb * bs + 64, np.uint8)
        c_dret = np.zeros(nb, np.int32)
        c_dcap = np.full(nb, bs, np.int32)
        tc = time.perf_counter()
        L.oracle_compress_linear_batch(host.ctypes.data, c_off.ctypes.data, c_len.ctypes.data,
                                       c_tt.ctypes.data, c_out.ctypes.data, c_doff.ctypes.data,
                                       c_cap.ctypes.data, c_ret.ctypes.data, nb, threads)
        tc = time.perf_counter() - tc
        td = time.perf_counter()
        L.oracle_decompress_batch(c_out.ctypes.data, c_doff.ctypes.data, c_ret.ctypes.data,
                                  c_dec.ctypes.data, c_off.ctypes.data, c_dcap.ctypes.data,
                                  c_dret.ctypes.data, nb, threads)
        td = time.perf_counter() - td
        if not (c_ret == rets[:nb]).all() or not (c_dret == bs).all():
            raise SystemExit("bench: CPU baseline disagrees with the GPU frames")
        ub = nb * bs
        result["cpu_baseline"] = {
            "value": round(ub / (tc + td) / 2**30, 4), "unit": "GiB/s", "cores": threads,
            "kind": "port",
            "sample": f"{nb} x {bs} B blocks of the same workload ({ub / 2**20:.0f} MiB), "
                      f"oracle/lz4e_oracle.c linear restatement, {threads} threads; "
                      f"compress {ub / tc / 2**30:.3f} GiB/s, decompress {ub / td / 2**30:.3f} GiB/s",
        }
        result["vs_cpu_baseline"] = round(value / result["cpu_baseline"]["value"], 2)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
