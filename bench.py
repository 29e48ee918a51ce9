#!/usr/bin/env python3
"""bench.py -- LZ4E scatter-gather block codec on MI355X (BASELINE.json metric).

Metric: GiB/s compress+decompress (round trip, whole job), 64 KiB blocks,
plus the ratio delta vs the reference: every frame of the run is compared
with the CPU oracle's (tests-only restatement of the reference, used here as
the checker) and the delta is computed from the two sets of sizes.

A step = one pass of the hot path over one batch of synthetic input already
resident in HBM: LZ4E compress of every block (one launch), then LZ4E safe
decompress of every frame (one launch).  value = uncompressed bytes of all
ranks / max-over-ranks step time.

Default workload (configs[1] of BASELINE.json): Silesia-proxy, 3234 blocks of
64 KiB (~212 MB, the Silesia size) per GPU, each block a 16 x 4 KiB bio_vec
list (byU16 hash table).  Other workloads (--workload) are the parity
configurations: fio4k (configs[2]), sg512 (configs[3], byU32), text256k
(configs[4]; its line adds ``decompress_only``, the frames decoded alone as
that configuration asks, weak and strong over the ranks).

Multi-GPU: ``python bench.py --gpus N`` starts N ranks itself (through
torch.distributed.run, before anything touches a GPU); under an external
launcher WORLD_SIZE must equal --gpus.  One rank per GPU, RCCL between them.
Two lines of the same run:
* ``value`` -- weak scaling: every rank its own Silesia-sized corpus (corpus
  multiplier k = N, stated in ``config``), no data-path collective;
* ``strong`` -- the one 3234-block corpus dealt over the N ranks as a chunk
  queue (lz4e_amd.shards.ChunkQueue): a calibration pass, an all_gather of
  {blocks_done, compressed_bytes, busy}, the chunk moves that even out the
  projected times sent rank to rank over RCCL, then the timed steps.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lz4-sgori_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

WORKLOADS = {
    # name: (block bytes, table class, generator, bio_vec segment bytes, description)
    "silesia64k": (65536, 1, "silesia", 4096,
                   "Silesia-proxy, 64 KiB independent blocks (16 x 4 KiB bio_vecs, byU16), round trip"),
    "fio4k": (4096, 1, "fio", 4096,
              "fio buffer_compress_percentage=50 pattern, 4 KiB chunks (1 x 4 KiB bio_vec, byU16), round trip"),
    "sg512": (65536, 3, "silesia", 512,
              "Silesia-proxy, 64 KiB blocks of 128 x 512 B bio_vecs (byU32), round trip"),
    "text256k": (262144, 3, "text", 262144,
                 "enwik9-proxy text, 256 KiB blocks (1 bio_vec, byU32), round trip"),
}
# configs[1]/[3]: the Silesia size (211,938,580 B) in 64 KiB blocks; configs[2]: 1 GiB of
# 4 KiB chunks; configs[4]: enwik9 (10^9 B) in 256 KiB blocks, the last one 182,784 B
DEFAULT_BLOCKS = {"silesia64k": 3234, "fio4k": 262144, "sg512": 3234, "text256k": 3815}
TOTAL_BYTES = {"text256k": 10**9}
CORPUS_SEED = 0x5157


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="silesia64k", choices=sorted(WORKLOADS))
    ap.add_argument("--blocks", type=int, default=0, help="blocks per GPU (0: workload default)")
    ap.add_argument("--chunk", type=int, default=16, help="blocks per chunk of the strong-scaling queue")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive chunk-layer run")
    ap.add_argument("--no-single-call", action="store_true", help="skip the single-call latency leg")
    ap.add_argument("--no-strong", action="store_true", help="skip the strong-scaling line")
    ap.add_argument("--no-parity", action="store_true", help="skip the every-frame oracle check")
    ap.add_argument("--no-decompress-only", action="store_true",
                    help="text256k: skip the decompress-only leg (configs[4])")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check only: start the ranks (gloo), report, touch no GPU")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> None:
    """--gpus N without a launcher: start N ranks under torch.distributed.run
    (this process has touched no GPU) and exit with their status."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None:
        if args.gpus > 1:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
                   f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
            env = dict(os.environ)
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            sys.exit(subprocess.run(cmd, env=env).returncode)
        return
    if int(world_env) != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={world_env} but --gpus {args.gpus}")


def host_cores() -> int:
    """CPU threads this process may use: its affinity mask, capped by a cgroup
    CPU quota and by OMP_NUM_THREADS when the host sets one.  (os.cpu_count()
    reports the whole machine; a shared GPU host gives each GPU a share.)"""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(p))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def make_data(gen: str, nbytes: int, seed: int) -> np.ndarray:
    from lz4e_amd import corpus
    if gen == "silesia":
        return corpus.silesia_proxy(nbytes, seed)
    if gen == "fio":
        return corpus.fio_pattern(nbytes, seed)
    return corpus.text_proxy(nbytes, seed)


class Batch:
    """Device-resident blocks of one size: input, frame slots, output."""

    def __init__(self, d_src, lens, bs: int, cls: int, dev):
        import torch
        lens = np.asarray(lens, dtype=np.int64)
        nblk = len(lens)
        self.nblk, self.bs, self.cls, self.dev, self.lens = nblk, bs, cls, dev, lens
        self.U = int(lens.sum())
        self.max_cap = int(lens.max()) if nblk else 0
        self.offs = np.arange(nblk, dtype=np.int64) * bs
        self.cap1 = bs + bs // 255 + 16
        self.slot = (self.cap1 + 64 + 15) // 16 * 16
        self.doffs = np.arange(nblk, dtype=np.int64) * self.slot
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).to(dev)
        self.d_src = d_src
        self.d_off, self.d_len = t(self.offs, np.int64), t(lens, np.int32)
        self.d_tt = t(np.full(nblk, cls), np.uint8)
        self.d_dst = torch.zeros(nblk * self.slot, dtype=torch.uint8, device=dev)
        self.caps = lens + lens // 255 + 16
        self.d_doff, self.d_cap = t(self.doffs, np.int64), t(self.caps, np.int32)
        self.d_ret = torch.zeros(nblk, dtype=torch.int32, device=dev)
        self.d_out = torch.zeros(nblk * bs + 64, dtype=torch.uint8, device=dev)
        self.d_dret = torch.zeros(nblk, dtype=torch.int32, device=dev)
        self.stream = torch.cuda.current_stream(dev)

    def compress(self):
        import lz4e_amd
        lz4e_amd.compress_batch_dev(self.d_src, self.d_off, self.d_len, self.d_tt, self.d_dst,
                                    self.d_doff, self.d_cap, self.d_ret, max_len=self.bs,
                                    stream=self.stream.cuda_stream)

    def decompress(self):
        import lz4e_amd
        lz4e_amd.decompress_batch_dev(self.d_dst, self.d_doff, self.d_ret, self.d_out, self.d_off,
                                      self.d_len, self.d_dret, stream=self.stream.cuda_stream,
                                      max_cap=self.max_cap)

    def run(self, steps: int, timed: bool):
        """steps x (compress, decompress); -> (wall s, mean compress ms, mean decompress ms)."""
        import torch
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
               torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        for e0, e1, e2 in ev:
            e0.record(self.stream)
            self.compress()
            e1.record(self.stream)
            self.decompress()
            e2.record(self.stream)
        torch.cuda.synchronize(self.dev)
        wall = time.perf_counter() - t0
        comp = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))
        dec = float(np.mean([b.elapsed_time(c) for _, b, c in ev]))
        return wall, comp, dec

    def check_roundtrip(self) -> int:
        import torch
        rets = self.d_ret.cpu().numpy()
        n = self.U
        if (rets <= 0).any() or not torch.equal(self.d_out[:n], self.d_src[:n]) or \
                not (self.d_dret.cpu().numpy() == self.lens).all():
            raise SystemExit("bench: round trip mismatch")
        self.rets = rets
        return int(rets.astype(np.int64).sum())


def oracle_frames(host: np.ndarray, b: Batch, threads: int):
    """Every block through the oracle (compress, then decompress of its
    frames), timed.  -> (ret, frames buffer, compress s, decompress s)."""
    import oracle_ref
    L = oracle_ref.load()
    nb = b.nblk
    c_off = np.ascontiguousarray(b.offs.astype(np.uint64))
    c_len = np.ascontiguousarray(b.lens.astype(np.uint32))
    c_tt = np.full(nb, b.cls, np.uint8)
    c_cap = np.ascontiguousarray(b.caps.astype(np.uint32))
    c_doff = np.ascontiguousarray(b.doffs.astype(np.uint64))
    c_out = np.zeros(nb * b.slot, np.uint8)
    c_ret = np.zeros(nb, np.int32)
    c_dec = np.zeros(nb * b.bs + 64, np.uint8)
    c_dret = np.zeros(nb, np.int32)
    c_dcap = np.ascontiguousarray(b.lens.astype(np.int32))
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
    if not (c_dret == b.lens).all() or not np.array_equal(c_dec[:b.U], host[:b.U]):
        raise SystemExit("bench: oracle round trip failed")
    return c_ret, c_out, tc, td


def parity(host: np.ndarray, b: Batch, threads: int) -> dict:
    """Every GPU frame against the oracle's: sizes and bytes."""
    c_ret, c_out, tc, td = oracle_frames(host, b, threads)
    g_out = b.d_dst.cpu().numpy()
    g_ret = b.rets
    same_size = int((g_ret == c_ret).sum())
    same = 0
    for i in range(b.nblk):
        o, r = int(b.doffs[i]), int(g_ret[i])
        if r == c_ret[i] and np.array_equal(g_out[o:o + r], c_out[o:o + r]):
            same += 1
    U = b.U
    r_gpu = U / float(g_ret.astype(np.int64).sum())
    r_ref = U / float(c_ret.astype(np.int64).sum())
    return {"frames": b.nblk, "frames_identical": same, "sizes_identical": same_size,
            "ratio_gpu": r_gpu, "ratio_ref": r_ref, "ratio_delta": r_gpu - r_ref,
            "oracle_compress_s": tc, "oracle_decompress_s": td}


def end_to_end(host: np.ndarray, lens, bs: int, seg: int, reps: int = 3) -> dict:
    """lz4e_chunk_write_batch over the same blocks given as host bio_vec lists
    (seg-byte segments): SG gather -> H2D -> compress -> decompress -> D2H ->
    copy-out, four pipeline slots.  The host buffers are pageable numpy
    memory, as a bio's pages would be."""
    import ctypes

    import lz4e_amd
    lens = np.asarray(lens, dtype=np.int64)
    nblk = len(lens)
    U = int(lens.sum())
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
        its[i].bi_size = int(lens[i])
        reqs[i].src = ctypes.cast(bvp + i * nseg * ctypes.sizeof(lz4e_amd.BioVec),
                                  ctypes.POINTER(lz4e_amd.BioVec))
        reqs[i].srcIter = ctypes.pointer(its[i])
        reqs[i].data = out.ctypes.data + i * bs
    L = lz4e_amd.lib()
    times = []
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        good = L.lz4e_chunk_write_batch(reqs, nblk, None)
        times.append(time.perf_counter() - t0)
        if good != nblk:
            raise SystemExit(f"bench: chunk pipeline failed ({good}/{nblk}): {lz4e_amd.last_error()}")
    if not np.array_equal(out[:U], host[:U]):
        raise SystemExit("bench: chunk pipeline round trip mismatch")
    t = float(np.median(times[1:]))
    return {"value": round(U / t / 2**30, 3), "unit": "GiB/s", "ms": round(t * 1e3, 2),
            "path": f"lz4e_chunk_write_batch: {nblk} WRITE bios of {nseg} x {seg} B host segments, "
                    "SG gather -> H2D -> compress -> decompress -> D2H -> copy-out (PCIe-inclusive)"}


def single_call(threads_list=(1, 4, 16), calls: int = 400) -> dict:
    """configs[0]: one 4 KiB block (01.txt[0:4096], 1 x 4096 bio_vec) through
    the drop-in LZ4E_compress_default / LZ4E_decompress_safe, one synchronous
    call at a time as the chunk layer makes them (lz4e_chunk.c:139-159),
    from 1 and from T concurrent threads; beside the single-thread oracle on
    the same block (faithful SG walk and linear).  Timed through ctypes."""
    import ctypes
    import threading

    import lz4e_amd
    import oracle_ref
    from lz4e_amd import BYU16, compress_bound, make_sg
    data = open(os.path.join(REPO, "tests", "golden", "test_files", "01.txt"), "rb").read()[:4096]
    n, cap = len(data), compress_bound(4096)
    er, ef, _, _ = oracle_ref.compress(data, BYU16)
    L, O = lz4e_amd.lib(), oracle_ref.load()

    def worker(nc, lat_c, lat_d, errs):
        src = make_sg(data, [n])
        dst = make_sg(b"", [4096, cap - 4096], capacity=cap)
        wrk = (ctypes.c_uint8 * lz4e_amd.LZ4E_MEM_COMPRESS)()
        fsrc = ctypes.create_string_buffer(ef, len(ef))
        dout = ctypes.create_string_buffer(n + 16)
        for k in range(nc):
            src.it.bi_size, src.it.bi_idx, src.it.bi_bvec_done = n, 0, 0
            dst.it.bi_size, dst.it.bi_idx, dst.it.bi_bvec_done = cap, 0, 0
            t0 = time.perf_counter()
            r = L.LZ4E_compress_default(src.bvecs, dst.bvecs, ctypes.byref(src.it),
                                        ctypes.byref(dst.it), wrk)
            t1 = time.perf_counter()
            d = L.LZ4E_decompress_safe(fsrc, dout, len(ef), n)
            t2 = time.perf_counter()
            lat_c.append(t1 - t0)
            lat_d.append(t2 - t1)
            if k == nc - 1 and (r != er or dst.read_prefix(r) != ef or d != n or dout.raw[:n] != data):
                errs.append(k)

    res = {"block": "01.txt[0:4096], 1 x 4096 bio_vec, byU16, dst capacity 4128", "threads": {}}
    worker(20, [], [], [])  # warm the pool / first-launch costs
    for T in threads_list:
        lat_c, lat_d, errs = [], [], []
        th = [threading.Thread(target=worker, args=(calls, lat_c, lat_d, errs)) for _ in range(T)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        wall = time.perf_counter() - t0
        if errs:
            raise SystemExit("bench: single-call result differs from the oracle")
        res["threads"][str(T)] = {
            "compress_us_p50": round(float(np.percentile(lat_c, 50)) * 1e6, 1),
            "compress_us_p99": round(float(np.percentile(lat_c, 99)) * 1e6, 1),
            "decompress_us_p50": round(float(np.percentile(lat_d, 50)) * 1e6, 1),
            "decompress_us_p99": round(float(np.percentile(lat_d, 99)) * 1e6, 1),
            "round_trips_per_s": round(T * calls / wall, 1),
            "GiB_per_s": round(T * calls * n / wall / 2**30, 4),
        }
    # the oracle, one thread, same block
    src = make_sg(data, [n])
    dst = make_sg(b"", [4096, cap - 4096], capacity=cap)
    wrk = (ctypes.c_uint8 * lz4e_amd.LZ4E_MEM_COMPRESS)()
    sg_t, lin_t, dec_t = [], [], []
    ibuf = ctypes.create_string_buffer(data, n)
    obuf = ctypes.create_string_buffer(cap + 64)
    fsrc = ctypes.create_string_buffer(ef, len(ef))
    dout = ctypes.create_string_buffer(n + 64)
    for _ in range(200):
        src.it.bi_size, src.it.bi_idx, src.it.bi_bvec_done = n, 0, 0
        dst.it.bi_size, dst.it.bi_idx, dst.it.bi_bvec_done = cap, 0, 0
        t0 = time.perf_counter()
        O.oracle_compress_sg(src.bvecs, dst.bvecs, ctypes.byref(src.it), ctypes.byref(dst.it), wrk)
        t1 = time.perf_counter()
        O.oracle_compress_linear(ibuf, n, BYU16, obuf, cap, None, None)
        t2 = time.perf_counter()
        O.oracle_decompress_safe(fsrc, dout, len(ef), n)
        t3 = time.perf_counter()
        sg_t.append(t1 - t0)
        lin_t.append(t2 - t1)
        dec_t.append(t3 - t2)
    res["cpu_oracle_1thread"] = {
        "compress_sg_us_p50": round(float(np.median(sg_t)) * 1e6, 1),
        "compress_linear_us_p50": round(float(np.median(lin_t)) * 1e6, 1),
        "decompress_us_p50": round(float(np.median(dec_t)) * 1e6, 1),
    }
    return res


def block_floor(b: "Batch", top: int = 4, cands: int = 32, reps: int = 5) -> dict:
    """The per-block floor of a step: the slowest blocks' compress + decode
    time with the chip to themselves.  A stamped compress pass (per-block
    cycle counters, lz4e_debug_compress_stamped) names the `cands` blocks
    with the most cycles under the full launch; each is compressed alone
    once, stamped (its cycles with the chip to itself: a clock-free count,
    the same on every box), and the `top` slowest by that count are then
    compressed and decoded alone (one-block launches, HIP events on the
    batch's stream, each pair right after a full-batch compress so the lone
    wave runs at the clock the chip holds under this workload, median of
    `reps`).  Choosing by the lone count, not by the full-launch count (which
    moves with the launch's placement), keeps the chosen block the same from
    box to box.  However many GPUs share the corpus, a step cannot be shorter
    than this: strong scaling's ceiling is step(N=1) / floor."""
    import ctypes

    import torch

    import lz4e_amd
    L = lz4e_amd.lib()
    P = ctypes.c_void_p
    L.lz4e_debug_compress_stamped.argtypes = [P] * 8 + [ctypes.c_uint32, ctypes.c_uint32, P, P]
    dbg = torch.zeros(b.nblk * 16, dtype=torch.int64, device=b.dev)
    rc = L.lz4e_debug_compress_stamped(b.d_src.data_ptr(), b.d_off.data_ptr(), b.d_len.data_ptr(),
                                       b.d_tt.data_ptr(), b.d_dst.data_ptr(), b.d_doff.data_ptr(),
                                       b.d_cap.data_ptr(), b.d_ret.data_ptr(), b.nblk, b.bs,
                                       b.stream.cuda_stream, dbg.data_ptr())
    torch.cuda.synchronize(b.dev)
    if rc != 0:
        raise SystemExit("bench: stamped compress failed: " + lz4e_amd.last_error())
    cyc = dbg.view(b.nblk, 16)[:, :6].sum(1).cpu().numpy()
    one = torch.zeros(16, dtype=torch.int64, device=b.dev)
    lone = []
    for i in np.argsort(cyc)[::-1][:cands]:
        i = int(i)
        sl = slice(i, i + 1)
        # the block alone, stamped: its cycles with the chip to itself
        one.zero_()
        L.lz4e_debug_compress_stamped(b.d_src.data_ptr(), b.d_off[sl].data_ptr(), b.d_len[sl].data_ptr(),
                                      b.d_tt[sl].data_ptr(), b.d_dst.data_ptr(), b.d_doff[sl].data_ptr(),
                                      b.d_cap[sl].data_ptr(), b.d_ret[sl].data_ptr(), 1, b.bs,
                                      b.stream.cuda_stream, one.data_ptr())
        torch.cuda.synchronize(b.dev)
        lone.append((int(one[:6].sum().item()), i))
    lone.sort(reverse=True)
    worst = []
    for alone, i in lone[:top]:
        sl = slice(i, i + 1)
        tcs, tds = [], []
        for _ in range(reps):
            # a full-batch compress right before each timed pair: the lone
            # wave runs at the clock the chip holds under this workload, not
            # at an idle or boost clock of whatever ran before
            b.compress()
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(b.stream)
            lz4e_amd.compress_batch_dev(b.d_src, b.d_off[sl], b.d_len[sl], b.d_tt[sl], b.d_dst,
                                        b.d_doff[sl], b.d_cap[sl], b.d_ret[sl], max_len=b.bs,
                                        stream=b.stream.cuda_stream)
            e1.record(b.stream)
            lz4e_amd.decompress_batch_dev(b.d_dst, b.d_doff[sl], b.d_ret[sl], b.d_out, b.d_off[sl],
                                          b.d_len[sl], b.d_dret[sl], stream=b.stream.cuda_stream,
                                          max_cap=b.bs)
            e2.record(b.stream)
            torch.cuda.synchronize(b.dev)
            tcs.append(e0.elapsed_time(e1))
            tds.append(e1.elapsed_time(e2))
        tc, td = float(np.median(tcs)), float(np.median(tds))
        worst.append((tc + td, tc, td, i, int(cyc[i]), alone))
    # the shader clock the chip holds right after a full-batch compress:
    # delta s_memtime / delta s_memrealtime x 100 MHz in a one-wave probe
    # (MI355X_MICROARCH.md:503), median of `reps`
    L.lz4e_debug_clock_probe.argtypes = [P, P, ctypes.c_uint32]
    probe = torch.zeros(3, dtype=torch.int64, device=b.dev)
    clock = []
    for _ in range(reps):
        b.compress()
        if L.lz4e_debug_clock_probe(b.stream.cuda_stream, probe.data_ptr(), 1 << 20) != 0:
            break
        torch.cuda.synchronize(b.dev)
        mt, rt = (int(v) for v in probe[:2].cpu())
        if rt > 0:
            clock.append(mt / rt * 0.1)
    # restore the batch's frames (the single-block launches rewrote their own)
    b.compress()
    torch.cuda.synchronize(b.dev)
    worst.sort(reverse=True)
    t, tc, td, i, c, alone = worst[0]
    ghz = float(np.median(clock)) if clock else None
    return {"floor_ms": round(t, 4), "compress_ms": round(tc, 4), "decompress_ms": round(td, 4),
            "block": i, "stamped_cycles_in_full_launch": c, "stamped_cycles_alone": alone,
            "clock_ghz_est": round(ghz, 3) if ghz else None,
            "clock_ghz_runs": [round(x, 3) for x in clock],
            "stamped_ms_at_clock_est": round(alone / (ghz * 1e6), 4) if ghz else None,
            "max_stamped_cycles_alone": lone[0][0] if lone else None,
            "method": f"of the {cands} blocks with the most stamped compress cycles in the full launch, "
                      f"the {top} with the most stamped compress cycles alone (the decode leg plays no part "
                      f"in the choice), each compressed and decoded alone "
                      f"right after a full-batch compress (median of {reps}); the slowest sum (the "
                      f"unstamped kernels' HIP-event times) is the floor.  clock_ghz_est = delta "
                      f"s_memtime / delta s_memrealtime x 100 MHz of a one-wave probe launched right "
                      f"after a full-batch compress (median of {reps}); stamped_ms_at_clock_est = the "
                      f"stamped cycles alone at that clock (the stamped build runs ~11 % more cycles "
                      f"than the timed one, so it is not the floor's compress time)"}


def decompress_only(b: "Batch", steps: int, rank: int, world: int, dist, dev, traffic_json: str,
                    workload: str) -> dict:
    """configs[4] ("Decompress-only, enwik9 at 256 KiB blocks, 8 x MI355X"):
    the frames of the last compress, already in HBM, decoded alone -- `steps`
    timed launches between a barrier + synchronize on both sides, the max
    over ranks.  Two lines:
    * weak: every rank decodes all of its corpus (N corpora);
    * strong: the one job of b.nblk blocks dealt over the ranks as contiguous
      slices of the block list (rank r decodes blocks [r n/N, (r+1) n/N) of
      its corpus; same generator, so the slices are alike) -- blocks are
      independent, so there is no data-path collective.
    Roofline: algorithmic C + U bytes of one launch / its mean duration."""
    import torch
    import lz4e_amd
    from lz4e_amd.shards import reduce_step
    group = dist.group.WORLD if dist else None
    sizes = b.rets.astype(np.int64)

    def timed(sl) -> float:
        # every rank passes both barriers, an empty slice included
        args_ = (b.d_dst, b.d_doff[sl], b.d_ret[sl], b.d_out, b.d_off[sl], b.d_len[sl], b.d_dret[sl])
        n = sl.stop - sl.start

        def launch():
            if n > 0:
                lz4e_amd.decompress_batch_dev(*args_, stream=b.stream.cuda_stream, max_cap=b.max_cap)
        for _ in range(2):  # warm-up launches
            launch()
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(b.stream)
        for _ in range(steps):
            launch()
        e1.record(b.stream)
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        return e0.elapsed_time(e1) / steps if n > 0 else 0.0

    traffic = None
    if os.path.exists(traffic_json):
        try:
            traffic = json.load(open(traffic_json)).get(workload, {}).get("decompress")
        except (OSError, ValueError):
            traffic = None
    out = {"kernel": "decompress", "steps": steps}
    # weak: all blocks on every rank
    ms = timed(slice(0, b.nblk))
    if not (b.d_dret.cpu().numpy() == b.lens).all():
        raise SystemExit("bench: decompress-only leg decoded wrong sizes")
    (ms_max,), C_all = reduce_step([ms], int(sizes.sum()), group, dev)
    U, C = int(b.lens.sum()), int(sizes.sum())
    out["weak"] = {"value": round(U * world / (ms_max / 1e3) / 2**30, 3), "unit": "GiB/s",
                   "ms_per_step": round(ms_max, 4), "blocks_per_gpu": b.nblk,
                   "roofline": {"bound": "hbm", "achieved": round((U + C) / (ms / 1e3) / 1e9, 2),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": round((U + C) / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 5),
                                "traffic": traffic, "algorithmic_bytes_per_launch": U + C}}
    # strong: one job of b.nblk blocks over the ranks
    lo, hi = rank * b.nblk // world, (rank + 1) * b.nblk // world
    ms_s = timed(slice(lo, hi))
    (ms_s_max,), _ = reduce_step([ms_s], 0, group, dev)
    out["strong"] = {"value": round(U / (ms_s_max / 1e3) / 2**30, 3) if ms_s_max > 0 else None,
                     "unit": "GiB/s", "ms_per_step": round(ms_s_max, 4), "blocks_job": b.nblk,
                     "blocks_this_rank": hi - lo,
                     "note": "rank r decodes blocks [r n/N, (r+1) n/N) of its corpus (same generator)"}
    return out


def strong_scaling(args, rank, world, dist, dev, bs, cls, gen, threads) -> dict:
    """The one corpus of the default block count, dealt over the ranks as a
    chunk queue, calibrated, rebalanced over RCCL, then timed."""
    import torch

    from lz4e_amd.shards import ChunkQueue, reduce_step
    nblk_job = args.blocks or DEFAULT_BLOCKS[args.workload]
    q = ChunkQueue(nblk_job, args.chunk, rank, world)
    host_all = make_data(gen, nblk_job * bs, CORPUS_SEED)
    chunk_data = {}
    for c in q.queue:  # this rank's initial chunks only reach its HBM
        lo, hi = q.chunk_range(c)
        chunk_data[c] = torch.from_numpy(host_all[lo * bs:hi * bs].copy()).to(dev)
    del host_all
    group = dist.group.WORLD if dist else None

    def build():
        d_src = torch.cat([chunk_data[c] for c in q.queue]) if q.queue else \
            torch.zeros(0, dtype=torch.uint8, device=dev)
        return Batch(d_src, [bs] * len(q.blocks()), bs, cls, dev)

    b = build()
    if b.nblk:
        b.run(max(1, args.warmup), False)
        _, cm, dm = b.run(max(2, args.steps), False)
        busy = (cm + dm) / 1e3
        C = b.check_roundtrip()
    else:
        busy, C = 0.0, 0
    stats = q.progress(b.nblk, C, busy, group, dev)
    before = [s[2] * 1e3 for s in stats]
    moves = q.rebalance(stats, chunk_data, lambda c: (q.chunk_range(c)[1] - q.chunk_range(c)[0]) * bs,
                        group, dev)
    b = build()
    if b.nblk:
        b.run(1, False)
    if dist:
        dist.barrier()
    if b.nblk:
        wall, cm, dm = b.run(args.steps, True)
    else:
        torch.cuda.synchronize(dev)
        wall, cm, dm = 0.0, 0.0, 0.0
    if dist:
        dist.barrier()
    # every frame of this rank's chunks against the oracle
    C = b.check_roundtrip() if b.nblk else 0
    ok = 1
    if b.nblk and not args.no_parity:
        p = parity(b.d_src.cpu().numpy(), b, threads)
        ok = int(p["frames_identical"] == b.nblk)
    (step_s, cm_max, dm_max, busy_self), C_all = reduce_step(
        [wall / args.steps, cm, dm, (cm + dm)], C, group, dev)
    okv = torch.tensor([ok], dtype=torch.int64, device=dev)
    if dist:
        dist.all_reduce(okv, op=dist.ReduceOp.MIN)
    U_all = nblk_job * bs
    return {
        "scaling": "strong", "blocks": nblk_job, "chunk_blocks": args.chunk,
        "value": round(U_all / step_s / 2**30, 3), "unit": "GiB/s",
        "ms_per_step": round(step_s * 1e3, 3), "compress_ms_max": round(cm_max, 4),
        "decompress_ms_max": round(dm_max, 4), "ratio": round(U_all / C_all, 5),
        "calibration_busy_ms_per_rank": [round(x, 3) for x in before],
        "chunks_moved": len(moves), "blocks_on_this_rank0": b.nblk if rank == 0 else None,
        "frames_identical_to_oracle": bool(okv.item()),
    }


def main():
    args = parse()
    launch_ranks(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))

    if args.dry_run:
        import torch.distributed as dist
        if world > 1:
            dist.init_process_group("gloo")
            v = [None] * world
            dist.all_gather_object(v, {"rank": rank, "local_rank": local, "pid": os.getpid()})
            dist.destroy_process_group()
        else:
            v = [{"rank": 0, "local_rank": 0, "pid": os.getpid()}]
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": v}), flush=True)
        return

    import torch

    import lz4e_amd
    from lz4e_amd.shards import frame_layout, reduce_step
    sys.path.insert(0, os.path.join(REPO, "tests"))

    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)
    if not lz4e_amd.gpu_available():
        raise SystemExit("bench: HIP path unavailable: " + lz4e_amd.last_error())
    threads = args.cpu_threads or max(1, host_cores() // max(1, local_world))

    bs, cls, gen, seg, desc = WORKLOADS[args.workload]
    nblk = args.blocks or DEFAULT_BLOCKS[args.workload]
    U = min(nblk * bs, TOTAL_BYTES.get(args.workload, nblk * bs)) if not args.blocks else nblk * bs
    lens = np.full(nblk, bs, dtype=np.int64)
    lens[-1] = U - (nblk - 1) * bs
    host = np.zeros(nblk * bs, np.uint8)
    host[:U] = make_data(gen, U, CORPUS_SEED + 7919 * rank)
    b = Batch(torch.from_numpy(host).to(dev), lens, bs, cls, dev)

    b.run(max(1, args.warmup), False)
    C = b.check_roundtrip()

    # ---- timed region (weak scaling: every rank its own corpus) --------------
    if dist:
        dist.barrier()
    wall, comp_ms, dec_ms = b.run(args.steps, True)
    if dist:
        dist.barrier()
    step_s = wall / args.steps
    group = dist.group.WORLD if dist else None
    _, C_all, _ = frame_layout(C, nblk, group, dev)
    (step_s, comp_ms, dec_ms), _ = reduce_step([step_s, comp_ms, dec_ms], C, group, dev)
    U_all = U * world
    value = U_all / step_s / 2**30

    # ---- every frame against the oracle (the ratio delta is measured) --------
    par = None
    if not args.no_parity:
        par = parity(host, b, threads)
        if par["frames_identical"] != nblk:
            raise SystemExit(f"bench: {nblk - par['frames_identical']} frames differ from the oracle")

    # ---- roofline of the dominant kernel ---------------------------------------
    dom = "compress" if comp_ms >= dec_ms else "decompress"
    dom_ms = max(comp_ms, dec_ms)
    achieved = (U + C) / (dom_ms / 1e3) / 1e9  # algorithmic U + C bytes per launch
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            traffic = tj.get(args.workload, {}).get(dom)
        except (OSError, ValueError):
            traffic = None
    roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "algorithmic_bytes_per_launch": int(U + C),
                "other_kernel": {"kernel": "decompress" if dom == "compress" else "compress",
                                 "frac": round((U + C) / (min(comp_ms, dec_ms) / 1e3) / 1e9
                                               / HBM_PEAK_GBS, 5)}}

    result = {
        "metric": "GiB/s compress+decompress (whole node), 64 KiB blocks; ratio delta vs ref",
        "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": desc, "name": args.workload, "blocks_per_gpu": nblk,
                   "block_bytes": bs, "table_type": {1: "byU16", 3: "byU32", 7: "byU64"}[cls],
                   "bytes_per_gpu": U, "corpus_multiplier_k": world,
                   "parallelism": f"dp{world} (block shards, one corpus per rank)"},
        "ratio": round(U_all / C_all, 5),
        "ratio_delta_vs_ref": round(par["ratio_delta"], 6) if par else None,
        "parity": ({"frames_checked": par["frames"], "frames_identical": par["frames_identical"],
                    "ratio_ref_oracle": round(par["ratio_ref"], 5),
                    "note": "every frame of rank 0 vs the CPU oracle (reference restatement)"}
                   if par else None),
        "compress_ms": round(comp_ms, 4), "decompress_ms": round(dec_ms, 4),
        "compress_GiBps": round(U_all / (comp_ms / 1e3) / 2**30, 3),
        "decompress_GiBps": round(U_all / (dec_ms / 1e3) / 2**30, 3),
        "roofline": roofline,
    }

    # ---- configs[4]: decompress-only (the HBM-roofline stress run) -------------
    if args.workload == "text256k" and not args.no_decompress_only:
        result["decompress_only"] = decompress_only(b, args.steps, rank, world, dist, dev,
                                                    args.traffic_json, args.workload)

    # ---- strong scaling: one corpus over the N ranks (chunk queue) -------------
    if not args.no_strong:
        # the step's per-block floor (after the timed region; rank 0's corpus
        # is the N=1 corpus): the strong line cannot exceed step(N=1) / floor
        floor = block_floor(b) if rank == 0 else None
        if world > 1:
            result["strong"] = strong_scaling(args, rank, world, dist, dev, bs, cls, gen, threads)
        else:
            result["strong"] = {"scaling": "strong", "blocks": nblk, "value": round(value, 3),
                                "unit": "GiB/s", "ms_per_step": round(step_s * 1e3, 3),
                                "note": "N=1: the same corpus as value"}
        if floor is not None:
            result["strong"]["block_floor"] = floor
            # rank 0's weak-line step is one full corpus on one GPU: step(N=1)
            result["strong"]["ceiling_x"] = round(step_s * 1e3 / floor["floor_ms"], 3)

    # ---- end to end through the chunk layer (PCIe-inclusive, never `value`) ----
    if world == 1 and not args.no_e2e:
        result["end_to_end"] = end_to_end(host, lens, bs, seg)

    # ---- drop-in single calls (configs[0]) -------------------------------------
    if world == 1 and not args.no_single_call:
        result["single_call"] = single_call()

    # ---- CPU baseline (rank 0, N=1 only) ---------------------------------------
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle_ref
        if par is None:
            _, _, tc, td = oracle_frames(host, b, threads)
        else:
            tc, td = par["oracle_compress_s"], par["oracle_decompress_s"]
        result["cpu_baseline"] = {
            "value": round(U / (tc + td) / 2**30, 4), "unit": "GiB/s", "cores": threads,
            "kind": "port",
            "sample": f"all {nblk} x {bs} B blocks of the workload ({U / 2**20:.0f} MiB), "
                      f"oracle/lz4e_oracle.c linear restatement, {threads} threads (the host's CPU "
                      f"share); compress {U / tc / 2**30:.3f} GiB/s, decompress {U / td / 2**30:.3f} GiB/s",
        }
        # the faithful SG-walking compressor (the reference's per-access
        # bio_vec walk, lz4e_defs.h:352-585) on the same blocks; the
        # reference decompresses contiguous buffers, so its decode is the same
        L = oracle_ref.load()
        nb = nblk
        c_out = np.zeros(nb * b.slot, np.uint8)
        c_ret = np.zeros(nb, np.int32)
        ts = time.perf_counter()
        s_off = np.ascontiguousarray(b.offs.astype(np.uint64))
        s_len = np.ascontiguousarray(b.lens.astype(np.uint32))
        s_doff = np.ascontiguousarray(b.doffs.astype(np.uint64))
        s_cap = np.ascontiguousarray(b.caps.astype(np.uint32))
        L.oracle_compress_sg_batch(host.ctypes.data, s_off.ctypes.data, s_len.ctypes.data, seg,
                                   c_out.ctypes.data, s_doff.ctypes.data, s_cap.ctypes.data,
                                   c_ret.ctypes.data, nb, threads)
        ts = time.perf_counter() - ts
        if not (c_ret == b.rets).all():
            raise SystemExit("bench: SG oracle disagrees with the GPU frame sizes")
        result["cpu_baseline_sg"] = {
            "value": round(U / (ts + td) / 2**30, 4), "unit": "GiB/s", "cores": threads,
            "kind": "port",
            "sample": f"all {nblk} blocks as {bs // seg} x {seg} B bio_vecs through oracle_compress_sg "
                      f"(faithful SG walk), {threads} threads; compress {U / ts / 2**30:.4f} GiB/s, "
                      f"decompress (contiguous, as the reference) {U / td / 2**30:.3f} GiB/s",
        }
        result["vs_cpu_baseline"] = round(value / result["cpu_baseline"]["value"], 2)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
