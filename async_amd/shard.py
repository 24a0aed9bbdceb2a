"""Sharding independent stream buffers across the GPUs of one node.

SURVEY.md §8(e): buffers are independent, so a batch is split into
contiguous index ranges, one per rank, and each rank runs the batch kernels
on its own range with no data-path collective.  The single exchange step is
an all-gather of each rank's output byte total, which turns per-rank output
sizes into global output offsets (only needed when the results are laid out
as one logical array).  Decode output sizes depend on the data (the count
of alphabet characters), so that step cannot be precomputed for decoding.

Works with any torch.distributed backend: "nccl" (RCCL over xGMI) with CUDA
tensors on the GPU box, "gloo" with CPU tensors in the CPU tests.
"""
from __future__ import annotations

import bisect

import torch
import torch.distributed as dist


def by_index(nbuf: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced split of nbuf buffers: (first index, count)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    per, extra = divmod(nbuf, world)
    lo = rank * per + min(rank, extra)
    return lo, per + (1 if rank < extra else 0)


def by_bytes(lengths, world: int) -> list[int]:
    """Split points balancing payload bytes (ragged/Zipf batches).

    Returns world+1 buffer indices b[0]=0 <= ... <= b[world]=len(lengths);
    rank r owns buffers [b[r], b[r+1]).  Split r sits at the buffer boundary
    whose byte prefix is closest to r/world of the total, so every rank's
    load is within one buffer of the ideal.
    """
    n = len(lengths)
    prefix = [0]
    for x in lengths:
        prefix.append(prefix[-1] + int(x))
    total = prefix[-1]
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        i = bisect.bisect_left(prefix, target)  # prefix[i] >= target
        if i > 0 and target - prefix[i - 1] <= (prefix[i] - target if i <= n else 0):
            i -= 1
        bounds.append(min(n, max(bounds[-1], i)))
    bounds.append(n)
    return bounds


def exchange_totals(local_total: int, device=None) -> tuple[int, list[int]]:
    """The one collective: all-gather per-rank output byte totals.

    Returns (this rank's global output offset, all ranks' totals).
    Single-process (not initialised) -> (0, [local_total]).
    """
    if not dist.is_available() or not dist.is_initialized():
        return 0, [int(local_total)]
    world = dist.get_world_size()
    rank = dist.get_rank()
    if device is None:
        device = "cuda" if dist.get_backend() == "nccl" else "cpu"
    mine = torch.tensor([int(local_total)], dtype=torch.int64, device=device)
    allt = torch.zeros(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(allt, mine)
    totals = [int(v) for v in allt.cpu().tolist()]
    return sum(totals[:rank]), totals


def ranks_for(kernel_s: float, world: int, exchange_s: float, max_overhead: float = 0.1) -> int:
    """How many of `world` ranks a batch should be sharded over (SURVEY.md
    §8(e): shard "only when the batch is large enough to amortise").

    `kernel_s` is the batch's kernel time on one GPU (it splits evenly:
    the buffers are independent and resident per rank), `exchange_s` the
    one collective's latency (all-gather of a few bytes; `bench.py` measures
    it).  Each rank's share must keep the exchange within `max_overhead` of
    its own kernel time, so n <= kernel_s * max_overhead / exchange_s.
    Moving the buffers to the ranks first (root-scatter) never pays here:
    the transform runs faster than xGMI moves its bytes (`bench.py`'s
    root_scatter leg).
    """
    if world <= 1:
        return 1
    if exchange_s <= 0:  # a free exchange: every rank
        return world
    n = int(kernel_s * max_overhead / exchange_s)
    return max(1, min(world, n))

