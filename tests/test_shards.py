"""Multi-GPU bookkeeping (lz4e_amd.shards) on CPU: world_size-2 gloo.

The N>1 bench shards blocks across ranks with no data-path collective; the
collectives are the frame-stream layout (all_gather + exclusive scan) and the
max/sum step reduction.  Each rank here compresses its shard with the CPU
oracle (the checker stands in for the per-rank codec: no GPU on this host) and
the job's concatenated frame stream must equal the single-process one."""
import os
import socket

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
