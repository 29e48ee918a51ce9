"""Multi-GPU bookkeeping (lz4e_amd.shards) on CPU: world_size-2 gloo.

The N>1 bench shards blocks across ranks with no data-path collective; the
collectives are the frame-stream layout (all_gather + exclusive scan) and the
max/sum step reduction.  Each rank here compresses its shard with the CPU
oracle (the checker stands in for the per-rank codec: no GPU on this host) and
the job's concatenated frame stream must equal the single-process one."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lz4e_amd import BYU16, corpus
from lz4e_amd.shards import frame_layout, reduce_step, shard


def test_shard_partition():
    for n in (0, 1, 7, 64, 3234):
        for world in (1, 2, 3, 8):
            got = [shard(n, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            sizes = [hi - lo for lo, hi in got]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard(10, 2, 2)


def test_single_process_passthrough():
    assert frame_layout(123, 4) == (0, 123, 4)
    assert reduce_step([1.5, 2.0], 77) == ([1.5, 2.0], 77)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _blocks(n, bs=4096):
    data = corpus.silesia_proxy(n * bs, 0x5157, chunk=bs)
    return [data[i * bs:(i + 1) * bs].tobytes() for i in range(n)]


def _worker(rank, world, port, n_blocks, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle_ref
    lo, hi = shard(n_blocks, rank, world)
    frames = [oracle_ref.compress(b, BYU16)[1] for b in _blocks(n_blocks)[lo:hi]]
    local = b"".join(frames)
    base, total, nblk = frame_layout(len(local), hi - lo, dist.group.WORLD)
    times, csum = reduce_step([0.5 + rank, 2.0 - rank], len(local), dist.group.WORLD)
    with open(os.path.join(out_dir, f"r{rank}.bin"), "wb") as f:
        f.write(local)
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(f"{base} {total} {nblk} {times[0]} {times[1]} {csum}")
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_layout(tmp_path):
    import oracle_ref
    world, n = 2, 37
    mp.spawn(_worker, args=(world, _free_port(), n, str(tmp_path)), nprocs=world, join=True)
    ref = b"".join(oracle_ref.compress(b, BYU16)[1] for b in _blocks(n))
    stream = bytearray(len(ref))
    for r in range(world):
        base, total, nblk, t0, t1, csum = open(tmp_path / f"r{r}.txt").read().split()
        local = open(tmp_path / f"r{r}.bin", "rb").read()
        assert int(total) == len(ref) and int(nblk) == n and int(csum) == len(ref)
        assert (float(t0), float(t1)) == (1.5, 2.0)  # max over ranks
        stream[int(base):int(base) + len(local)] = local
    assert bytes(stream) == ref


# ---------------------------------------------------------------------------
# chunk queue + rebalance (north star: RCCL used only to rebalance the queue)
# ---------------------------------------------------------------------------

from lz4e_amd.shards import ChunkQueue, apply_moves, deal_chunks, rebalance_plan  # noqa: E402


def test_deal_chunks_round_robin():
    q = deal_chunks(10, 3)
    assert q == [[0, 3, 6, 9], [1, 4, 7], [2, 5, 8]]
    assert sorted(sum(q, [])) == list(range(10))


def test_rebalance_plan_evens_projected_time():
    queues = deal_chunks(40, 4)
    nb = [16] * 40
    busy = [4.0, 1.0, 1.0, 1.0]  # rank 0 four times slower per block
    moves = rebalance_plan(queues, nb, busy)
    assert moves and all(a == 0 for _, a, _ in moves)
    q2 = apply_moves(queues, moves)
    assert sorted(sum(q2, [])) == list(range(40))
    rate = [10 * 16 / b for b in busy]
    before = max(len(q) * 16 / r for q, r in zip(queues, rate))
    after = max(len(q) * 16 / r for q, r in zip(q2, rate))
    assert after < 0.5 * before
    # balanced input: nothing moves; the plan is deterministic
    assert rebalance_plan(queues, nb, [1.0] * 4) == []
    assert rebalance_plan(queues, nb, busy) == moves


def test_rebalance_plan_idle_rank():
    # a rank with no chunks (more ranks than chunks) pulls work, never gives any
    queues = deal_chunks(3, 4)
    assert queues[3] == []
    moves = rebalance_plan(queues, [16, 16, 16], [1.0, 1.0, 1.0, 0.0])
    assert all(b != 3 or a != 3 for _, a, b in moves)


def _rebalance_worker(rank, world, port, n_blocks, chunk, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle_ref
    bs = 4096
    q = ChunkQueue(n_blocks, chunk, rank, world)
    data = corpus.silesia_proxy(n_blocks * bs, 0x5157, chunk=bs)
    held = {}
    for c in q.queue:  # only this rank's initial chunks are materialised here
        lo, hi = q.chunk_range(c)
        held[c] = torch.from_numpy(data[lo * bs:hi * bs].copy())
    del data
    # calibration: rank 0 reports itself 3x slower per block -> it gives chunks away
    nb = len(q.blocks())
    stats = q.progress(nb, 0, (3.0 if rank == 0 else 1.0) * nb, dist.group.WORLD)
    moves = q.rebalance(stats, held, lambda c: (q.chunk_range(c)[1] - q.chunk_range(c)[0]) * bs,
                        dist.group.WORLD)
    assert sorted(held) == sorted(q.queue)
    frames = {}
    for c in q.queue:
        lo, hi = q.chunk_range(c)
        buf = held[c].numpy()
        for k, blk in enumerate(range(lo, hi)):
            frames[blk] = oracle_ref.compress(buf[k * bs:(k + 1) * bs].tobytes(), BYU16)[1]
    with open(os.path.join(out_dir, f"q{rank}.txt"), "w") as f:
        f.write(" ".join(f"{b}:{len(frames[b])}" for b in sorted(frames)) + "\n")
        f.write(" ".join(f"{c},{a},{b}" for c, a, b in moves))
    with open(os.path.join(out_dir, f"q{rank}.bin"), "wb") as f:
        f.write(b"".join(frames[b] for b in sorted(frames)))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_rebalance(tmp_path):
    """The calibrated rebalance moves chunks (payload over point-to-point
    send/recv) and the job's frames, reassembled in block order, equal the
    single-process stream."""
    import oracle_ref
    world, n, chunk = 2, 45, 4
    mp.spawn(_rebalance_worker, args=(world, _free_port(), n, chunk, str(tmp_path)), nprocs=world,
             join=True)
    frames = {}
    moves_seen = []
    for r in range(world):
        head, mv = open(tmp_path / f"q{r}.txt").read().split("\n")
        blob = open(tmp_path / f"q{r}.bin", "rb").read()
        pos = 0
        for tok in head.split():
            b, ln = map(int, tok.split(":"))
            assert b not in frames
            frames[b] = blob[pos:pos + ln]
            pos += ln
        moves_seen.append(mv)
    assert moves_seen[0] == moves_seen[1] and moves_seen[0]  # same plan everywhere, non-empty
    assert all(m.split(",")[1] == "0" for m in moves_seen[0].split())
    assert sorted(frames) == list(range(n))
    data = corpus.silesia_proxy(n * 4096, 0x5157, chunk=4096)
    ref = [oracle_ref.compress(data[i * 4096:(i + 1) * 4096].tobytes(), BYU16)[1] for i in range(n)]
    assert [frames[i] for i in range(n)] == ref


def test_bench_launches_ranks():
    """bench.py --gpus 2 starts two ranks itself (launcher check, no GPU)."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry-run"],
                         capture_output=True, text=True, timeout=180, env=env, check=True).stdout
    line = [x for x in out.splitlines() if x.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2 and sorted(r["rank"] for r in res["ranks"]) == [0, 1]
    env["WORLD_SIZE"] = "3"
    bad = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry-run"],
                         capture_output=True, text=True, timeout=60, env=env)
    assert bad.returncode != 0 and "WORLD_SIZE" in bad.stderr


def test_rebalance_plan_moves_each_chunk_once():
    """3, 4 and 8 ranks, uneven busy times: no chunk appears twice in a plan
    (a chunk relayed through a middle rank would be forwarded, in the same
    batch of point-to-point transfers, before it had arrived: ADVICE r02),
    the plan is a permutation of the chunks, and it never raises the
    projected slowest rank."""
    import random
    rng = random.Random(20260517)
    for _ in range(4000):
        world = rng.choice([3, 4, 8])
        n = rng.randint(world, 96)
        queues = deal_chunks(n, world)
        nb = [16] * n
        nb[-1] = rng.randint(1, 16)
        busy = [rng.uniform(0.5, 2.0) * sum(nb[c] for c in q) for q in queues]
        moves = rebalance_plan(queues, nb, busy)
        moved = [c for c, _, _ in moves]
        assert len(moved) == len(set(moved))
        q2 = apply_moves(queues, moves)
        assert sorted(sum(q2, [])) == list(range(n))
        rate = [sum(nb[c] for c in q) / b for q, b in zip(queues, busy)]
        proj = lambda qs: max(sum(nb[c] for c in q) / r for q, r in zip(qs, rate))
        assert proj(q2) <= proj(queues) + 1e-12
        # every move leaves its chunk's original owner
        assert all(c in queues[a] for c, a, _ in moves)


def _strong_worker(rank, world, port, n_blocks, chunk, out_dir):
    """The calls bench.strong_scaling makes, in its order (ChunkQueue ->
    progress -> rebalance -> rebuild from the held chunks), with the
    calibration busy time measured: the oracle compressing this rank's
    chunks.  Rank 0's blocks are text (slow to compress), rank 1's are
    incompressible bytes (the search skips ahead): two block classes."""
    import time
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle_ref
    bs = 4096
    q = ChunkQueue(n_blocks, chunk, rank, world)
    text = corpus.text_proxy(n_blocks * bs, 11)
    rnd = np.random.default_rng(12).integers(0, 256, n_blocks * bs, dtype=np.uint8)
    owner0 = set(deal_chunks(q.n_chunks, world)[0])

    def payload(c):
        lo, hi = q.chunk_range(c)
        src = text if c in owner0 else rnd
        return torch.from_numpy(src[lo * bs:hi * bs].copy())

    held = {c: payload(c) for c in q.queue}
    t0 = time.perf_counter()
    for _ in range(3):
        for c in q.queue:
            buf = held[c].numpy()
            for k in range(len(buf) // bs):
                oracle_ref.compress(buf[k * bs:(k + 1) * bs].tobytes(), BYU16)
    busy = time.perf_counter() - t0
    stats = q.progress(len(q.blocks()), 0, busy, dist.group.WORLD)
    moves = q.rebalance(stats, held, lambda c: (q.chunk_range(c)[1] - q.chunk_range(c)[0]) * bs,
                        dist.group.WORLD)
    assert sorted(held) == sorted(q.queue)
    out = {}
    for c in q.queue:
        assert torch.equal(held[c], payload(c))  # every received payload is the chunk's bytes
        lo, hi = q.chunk_range(c)
        buf = held[c].numpy()
        for k, blk in enumerate(range(lo, hi)):
            out[blk] = oracle_ref.compress(buf[k * bs:(k + 1) * bs].tobytes(), BYU16)[1]
    with open(os.path.join(out_dir, f"s{rank}.txt"), "w") as f:
        f.write(" ".join(f"{x:.6f}" for _, _, x in stats) + "\n")
        f.write(" ".join(f"{c},{a},{b}" for c, a, b in moves) + "\n")
        f.write(" ".join(f"{b}:{out[b].hex()}" for b in sorted(out)))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_strong_scaling_calls(tmp_path):
    """ChunkQueue through bench.strong_scaling's calls with measured
    calibration of two block classes: the plan is the same on both ranks,
    moves chunks only off the slower (text) rank, and the job's frames
    equal the single-process ones."""
    import oracle_ref
    world, n, chunk = 2, 48, 4
    mp.spawn(_strong_worker, args=(world, _free_port(), n, chunk, str(tmp_path)), nprocs=world,
             join=True)
    lines = [open(tmp_path / f"s{r}.txt").read().split("\n") for r in range(world)]
    assert lines[0][0] == lines[1][0] and lines[0][1] == lines[1][1]
    busy = [float(x) for x in lines[0][0].split()]
    assert busy[0] > busy[1]  # text compresses slower than incompressible bytes
    moves = [tuple(map(int, m.split(","))) for m in lines[0][1].split()]
    assert moves and all(a == 0 and b == 1 for _, a, b in moves)
    frames = {}
    for r in range(world):
        for tok in lines[r][2].split():
            b, h = tok.split(":")
            assert int(b) not in frames
            frames[int(b)] = bytes.fromhex(h)
    assert sorted(frames) == list(range(n))
    bs = 4096
    text = corpus.text_proxy(n * bs, 11)
    rnd = np.random.default_rng(12).integers(0, 256, n * bs, dtype=np.uint8)
    owner0 = set(deal_chunks(-(-n // chunk), world)[0])
    for b in range(n):
        src = text if b // chunk in owner0 else rnd
        assert frames[b] == oracle_ref.compress(src[b * bs:(b + 1) * bs].tobytes(), BYU16)[1]


def _donly_worker(rank, world, port, nblk, out_dir):
    """bench.decompress_only on `world` gloo ranks with the GPU calls faked
    (the decode fills its size slots; events report 1 ms): every rank passes
    the same barriers -- a rank whose strong slice is empty included -- and
    all ranks report the same max-over-ranks lines."""
    import json
    import types
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import lz4e_amd

    class Ev:
        def __init__(self, enable_timing=True):
            pass

        def record(self, stream=None):
            pass

        def elapsed_time(self, other):
            return 1.0 * (1 + rank)  # rank r is (r + 1)x slower

    torch.cuda.Event = Ev
    torch.cuda.synchronize = lambda *a, **k: None
    calls = []

    def fake_decode(src, src_off, src_len, dst, dst_off, dst_cap, ret, stream=None, max_cap=None):
        calls.append(int(src_len.numel()))
        ret.copy_(dst_cap)

    lz4e_amd.decompress_batch_dev = fake_decode
    lens = np.full(nblk, 1000, dtype=np.int64)
    t = lambda a, dt: torch.from_numpy(np.asarray(a).astype(dt))
    b = types.SimpleNamespace(
        nblk=nblk, lens=lens, rets=np.full(nblk, 400, dtype=np.int32), max_cap=1000,
        d_dst=torch.zeros(1), d_out=torch.zeros(1), stream=types.SimpleNamespace(cuda_stream=0),
        d_doff=t(np.zeros(nblk), np.int64), d_ret=t(np.full(nblk, 400), np.int32),
        d_off=t(np.zeros(nblk), np.int64), d_len=t(lens, np.int32), d_dret=t(np.zeros(nblk), np.int32))
    out = bench.decompress_only(b, 3, rank, world, dist, torch.device("cpu"), "", "text256k")
    out["calls"] = calls
    with open(os.path.join(out_dir, f"d{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_decompress_only_leg(tmp_path):
    """configs[4]'s decompress-only leg over two ranks, one block: rank 0's
    strong slice is empty (no launch) and rank 1 decodes the block; both
    reach the end, the weak and strong lines are the max over ranks."""
    import json
    world = 2
    mp.spawn(_donly_worker, args=(world, _free_port(), 1, str(tmp_path)), nprocs=world, join=True)
    r = [json.load(open(tmp_path / f"d{k}.json")) for k in range(world)]
    assert r[0]["weak"] == r[1]["weak"] and r[0]["strong"]["value"] == r[1]["strong"]["value"]
    assert r[0]["weak"]["ms_per_step"] == round(2.0 / 3, 4)  # max over ranks: 2 ms / 3 steps
    assert [x["strong"]["blocks_this_rank"] for x in r] == [0, 1]
    # weak: 2 warm-up + 3 timed launches of the whole batch on each rank;
    # strong: none on the empty rank, 5 of one block on the other
    assert r[0]["calls"] == [1] * 5 and r[1]["calls"] == [1] * 10
