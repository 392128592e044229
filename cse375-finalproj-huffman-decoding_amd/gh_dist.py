"""Multi-GPU plumbing for the sharded decode: one process per GPU, torch.distributed.

The compressed stream shards by gap-array segment boundaries: rank k
decodes segments [bounds[k], bounds[k+1]) of the SAME stream with no data-path
collective — each shard's first start bit comes from its own gap nibble, so the
only cross-shard fact is the output byte offset, which is an exclusive scan of the
per-shard symbol counts.  The reference has no multi-GPU path (its launcher is
single-device, decoder.cu:732-815); the north star adds an RCCL gather of the
decoded shards to one rank as the last step, timed separately from the decode.

Backend-agnostic: RCCL ("nccl") on the GPU box, gloo in the CPU tests.
"""
from __future__ import annotations

import time
from typing import List, Optional, Tuple

import gaphuff as gh


def shard_range(g: int, world: int, rank: int) -> Tuple[int, int]:
    """Segments [begin, end) of rank `rank` (gh_plan_shards: near-equal segment counts)."""
    b = gh.plan_shards(g, world)
    return b[rank], b[rank + 1]


def shard_alg_bytes(w: int, begin: int, end: int, out_bytes: int) -> int:
    """Algorithmic HBM bytes of one shard decode: payload words [4b, min(4e+1, W)),
    gap words [b/8, ceil(e/8)) and the decoded bytes written."""
    pay = max(0, min(4 * end + 1, w) - 4 * begin)
    gaps = (end + 7) // 8 - begin // 8
    return 4 * pay + 4 * gaps + out_bytes


def exclusive_offsets(dist, count: int, device) -> Tuple[int, List[int]]:
    """Output byte offset of this rank's shard (exclusive scan of shard sizes) and
    the list of all shard sizes, via one all_gather of one integer per rank."""
    import torch

    t = torch.tensor([count], dtype=torch.int64, device=device)
    allv = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(allv, t)
    sizes = [int(x.item()) for x in allv]
    rank = dist.get_rank()
    return sum(sizes[:rank]), sizes


def gather_to_root(dist, shard, nbytes: int, device) -> Tuple[Optional["torch.Tensor"], float]:
    """Gather every rank's decoded shard (uint8 tensor, first `nbytes` valid) to rank 0.

    Returns (concatenated output on rank 0 / None elsewhere, elapsed ms of the
    collective).  Shards are padded to the largest shard so one gather moves them."""
    import torch

    _, sizes = exclusive_offsets(dist, nbytes, device)
    cap = max(1, max(sizes))
    padded = torch.zeros(cap, dtype=torch.uint8, device=device)
    if nbytes:
        padded[:nbytes] = shard[:nbytes]
    rank, world = dist.get_rank(), dist.get_world_size()
    bufs = [torch.empty(cap, dtype=torch.uint8, device=device) for _ in range(world)] \
        if rank == 0 else None
    dist.barrier()
    if device is not None and torch.device(device).type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    dist.gather(padded, bufs, dst=0)
    if device is not None and torch.device(device).type == "cuda":
        torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    if rank != 0:
        return None, ms
    return torch.cat([bufs[k][:sizes[k]] for k in range(world)]), ms


def reduce_max_sum(dist, values: List[float], device) -> Tuple[List[float], List[float]]:
    """Element-wise MAX and SUM of per-rank float values."""
    import torch

    v = torch.tensor(values, dtype=torch.float64, device=device)
    if dist is None:
        return list(map(float, v)), list(map(float, v))
    mx, sm = v.clone(), v.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    return [float(x) for x in mx], [float(x) for x in sm]


def all_true(dist, ok: bool, device) -> bool:
    import torch

    if dist is None:
        return ok
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())
