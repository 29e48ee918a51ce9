"""Block sharding and chunk-queue rebalancing across the GPUs of one node
(SURVEY.md §8e).

Every LZ4E block is independent (the compressor memsets its state per call,
/root/reference/lz4e/lz4e_compress.c:548, and no dictionary is used), so a
job's blocks are dealt to ranks with no collective on the data path.  The
collectives are small and off the kernels' critical path:

* ``frame_layout``: one all_gather of the per-rank compressed byte counts
  (and block counts) -> each rank's base offset in the job's concatenated
  frame stream (an exclusive scan) and the job total;
* ``reduce_step``: max over ranks of the step times (the whole-job time is
  the slowest rank's) and sum of the compressed bytes;
* the chunk queue (:class:`ChunkQueue`): the job's blocks in fixed-size
  chunks, dealt round robin (block classes differ a lot in cost, and a
  contiguous deal can hand one rank all the slow ones).  After a calibration
  pass every rank all_gathers its ``{blocks_done, compressed_bytes,
  busy_us}``; all ranks then derive the same move plan
  (:func:`rebalance_plan`: chunks from the tail of the most loaded queue to
  the least loaded one while that lowers the projected slowest rank), and the
  moved chunks' input bytes travel rank to rank with point-to-point
  send/recv -- RCCL over xGMI on the GPU bench, gloo in the CPU tests.

The functions take a ``torch.distributed`` process group or ``None`` for a
single process.
"""
from typing import Dict, List, Optional, Sequence, Tuple

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


# ---------------------------------------------------------------------------
# chunk queue
# ---------------------------------------------------------------------------

def deal_chunks(n_chunks: int, world: int) -> List[List[int]]:
    """Initial queues: chunk c goes to rank c % world (in chunk order)."""
    return [list(range(r, n_chunks, world)) for r in range(world)]


def rebalance_plan(queues: Sequence[Sequence[int]], chunk_blocks: Sequence[int],
                   busy: Sequence[float], max_moves: int = 1 << 20) -> List[Tuple[int, int, int]]:
    """Moves (chunk, from_rank, to_rank) that even out the projected times.

    Rank r did ``sum(chunk_blocks[c] for c in queues[r])`` blocks in
    ``busy[r]`` seconds (its calibration pass), i.e. at rate
    blocks / busy.  Repeatedly the tail chunk of the rank with the largest
    projected time moves to the rank with the smallest one, as long as that
    lowers the larger of the two projected times.  Deterministic: every rank
    computes the same plan from the same all_gathered numbers.

    A chunk moves at most once: a received chunk is appended to its new
    rank's queue but never given away again (the payload exchange is one
    batch of point-to-point transfers, so a chunk relayed through a middle
    rank would be forwarded before it had arrived).  The chunk taken from the
    most loaded rank is the last one it held from the start.
    """
    world = len(queues)
    q = [list(x) for x in queues]
    blocks = [sum(chunk_blocks[c] for c in x) for x in q]
    rate = []
    for r in range(world):
        rate.append(blocks[r] / busy[r] if busy[r] > 0 and blocks[r] > 0 else None)
    known = [x for x in rate if x]
    if not known:
        return []
    fallback = sum(known) / len(known)
    rate = [x if x else fallback for x in rate]
    proj = [blocks[r] / rate[r] for r in range(world)]
    moves: List[Tuple[int, int, int]] = []
    moved = set()
    while len(moves) < max_moves:
        hi = max(range(world), key=lambda r: (proj[r], -r))
        lo = min(range(world), key=lambda r: (proj[r], r))
        if hi == lo:
            break
        own = [i for i, x in enumerate(q[hi]) if x not in moved]
        if not own:
            break
        c = q[hi][own[-1]]
        nb = chunk_blocks[c]
        new_hi = proj[hi] - nb / rate[hi]
        new_lo = proj[lo] + nb / rate[lo]
        if max(new_hi, new_lo) >= proj[hi]:
            break
        del q[hi][own[-1]]
        q[lo].append(c)
        moved.add(c)
        proj[hi], proj[lo] = new_hi, new_lo
        moves.append((c, hi, lo))
    return moves


def apply_moves(queues: Sequence[Sequence[int]], moves) -> List[List[int]]:
    q = [list(x) for x in queues]
    for c, a, b in moves:
        q[a].remove(c)
        q[b].append(c)
    return q


class ChunkQueue:
    """This rank's queue of chunks of a job of ``n_blocks`` blocks.

    ``chunk`` blocks per chunk (the last chunk may be shorter); ``queue`` is
    the list of chunk ids this rank owns, in processing order.
    """

    def __init__(self, n_blocks: int, chunk: int, rank: int, world: int):
        if chunk <= 0:
            raise ValueError("chunk must be positive")
        self.n_blocks, self.chunk, self.rank, self.world = n_blocks, chunk, rank, world
        self.n_chunks = -(-n_blocks // chunk)
        self.queues = deal_chunks(self.n_chunks, world)

    @property
    def queue(self) -> List[int]:
        return self.queues[self.rank]

    def chunk_range(self, c: int) -> Tuple[int, int]:
        lo = c * self.chunk
        return lo, min(self.n_blocks, lo + self.chunk)

    def chunk_blocks(self) -> List[int]:
        return [self.chunk_range(c)[1] - self.chunk_range(c)[0] for c in range(self.n_chunks)]

    def blocks(self) -> List[int]:
        """Global block ids of this rank's queue, in queue order."""
        out: List[int] = []
        for c in self.queue:
            lo, hi = self.chunk_range(c)
            out.extend(range(lo, hi))
        return out

    def progress(self, blocks_done: int, compressed_bytes: int, busy_s: float, group=None,
                 device: Optional[torch.device] = None) -> List[Tuple[int, int, float]]:
        """all_gather of every rank's ``{blocks_done, compressed_bytes, busy}``."""
        if group is None:
            return [(int(blocks_done), int(compressed_bytes), float(busy_s))]
        import torch.distributed as dist
        v = torch.tensor([blocks_done, compressed_bytes, int(round(busy_s * 1e9))],
                         dtype=torch.int64, device=device)
        allv = [torch.zeros_like(v) for _ in range(self.world)]
        dist.all_gather(allv, v, group=group)
        return [(int(t[0]), int(t[1]), int(t[2]) / 1e9) for t in allv]

    def rebalance(self, stats: Sequence[Tuple[int, int, float]], chunk_data: Dict[int, torch.Tensor],
                  chunk_nbytes, group=None, device: Optional[torch.device] = None,
                  max_moves: int = 1 << 20) -> List[Tuple[int, int, int]]:
        """Plan from the all_gathered ``stats`` and move chunk payloads.

        ``chunk_data`` maps each chunk this rank holds to its uint8 payload
        (on ``device``); ``chunk_nbytes(c)`` is chunk c's payload size (every
        rank can compute it).  Chunks this rank gives away are dropped from
        ``chunk_data``; chunks it receives are added.  Returns the moves.
        """
        moves = rebalance_plan(self.queues, self.chunk_blocks(), [s[2] for s in stats], max_moves)
        if not moves:
            return []
        if group is not None:
            import torch.distributed as dist
            ops = []
            for c, a, b in moves:
                if a == self.rank:
                    ops.append(dist.P2POp(dist.isend, chunk_data[c].contiguous(), b, group))
                elif b == self.rank:
                    buf = torch.empty(int(chunk_nbytes(c)), dtype=torch.uint8, device=device)
                    chunk_data[c] = buf
                    ops.append(dist.P2POp(dist.irecv, buf, a, group))
            if ops:
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
            for c, a, _ in moves:
                if a == self.rank:
                    chunk_data.pop(c, None)
        self.queues = apply_moves(self.queues, moves)
        return moves
