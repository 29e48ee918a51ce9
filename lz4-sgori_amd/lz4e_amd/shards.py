"""Block sharding across the GPUs of one node.

Every LZ4E block is independent (the compressor memsets its state per call,
/root/reference/lz4e/lz4e_compress.c:548, and no dictionary is used), so a
job of N blocks is split into contiguous shards, one per rank, with no
collective on the data path.  The only collectives are bookkeeping:

* ``frame_layout``: one all_gather of the per-rank compressed byte counts
  (and block counts) -> each rank's base offset in the job's concatenated
  frame stream (an exclusive scan) and the job total;
* ``reduce_step``: max over ranks of the step times (the whole-job time is
  the slowest rank's) and sum of the compressed bytes.

The functions take a ``torch.distributed`` process group (RCCL on the GPU
bench, gloo in the CPU tests) or ``None`` for a single process.
"""
from typing import Optional, Sequence, Tuple

import torch


def shard(n_blocks: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) block range of ``rank``; shard sizes differ by at most 1."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(n_blocks, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def frame_layout(local_bytes: int, local_blocks: int, group=None,
                 device: Optional[torch.device] = None) -> Tuple[int, int, int]:
    """-> (this rank's byte offset in the job's frame stream, total bytes, total blocks)."""
    if group is None:
        return 0, int(local_bytes), int(local_blocks)
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    v = torch.tensor([local_bytes, local_blocks], dtype=torch.int64, device=device)
    allv = [torch.zeros_like(v) for _ in range(world)]
    dist.all_gather(allv, v, group=group)
    sizes = [int(t[0]) for t in allv]
    return sum(sizes[:rank]), sum(sizes), sum(int(t[1]) for t in allv)


def reduce_step(times: Sequence[float], compressed_bytes: int, group=None,
                device: Optional[torch.device] = None) -> Tuple[list, int]:
    """-> (max over ranks of each time, sum over ranks of the compressed bytes)."""
    if group is None:
        return list(times), int(compressed_bytes)
    import torch.distributed as dist
    mx = torch.tensor(list(times), dtype=torch.float64, device=device)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    sm = torch.tensor([float(compressed_bytes)], dtype=torch.float64, device=device)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM, group=group)
    return [float(x) for x in mx.tolist()], int(sm.item())
