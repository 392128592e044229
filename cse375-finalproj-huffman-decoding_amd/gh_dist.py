"""Multi-GPU plumbing for the sharded decode: one process per GPU, torch.distributed.

The compressed stream shards by gap-array segment boundaries: rank k
decodes segments [bounds[k], bounds[k+1]) of the SAME stream with no data-path
collective — each shard's first start bit comes from its own gap nibble, so the
only cross-shard fact is the output byte offset, which is an exclusive scan of the
per-shard symbol counts.  The reference has no multi-GPU path (its launcher is
single-device, decoder.cu:732-815); the north star adds an RCCL gather of the
decoded shards to one rank as the last step, timed separately from the decode.

One stream, many readers: rank 0 builds the compressed.huff once and writes it to a
file (``share_stream``); every rank then streams only its own shard's words from that
file (``gh_ctx_load_file``), so no rank holds the global stream in memory.

Backend-agnostic: RCCL ("nccl") on the GPU box, gloo in the CPU tests.
"""
from __future__ import annotations

import os
import time
from typing import Callable, List, Optional, Tuple

import numpy as np

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


def _bcast_ints(dist, vals: List[int], device) -> List[int]:
    import torch

    t = torch.tensor(vals, dtype=torch.int64, device=device)
    if dist is not None:
        dist.broadcast(t, src=0)
    return [int(x) for x in t.cpu()]


def share_stream(dist, rank: int, path: str, make_image: Callable[[], np.ndarray],
                 device) -> dict:
    """Rank 0 builds the compressed.huff image (``make_image()``) and writes it to
    `path`; every rank gets the header sizes.  Returns {n, w, g, version, file_bytes}.

    The image goes to a temporary name first and is renamed when complete, so a reader
    never sees a partial file.  Callers remove `path` after every rank has loaded."""
    hdr = [0, 0, 0, 0, 0, 0]  # ok, n, w, g, version, file_bytes
    if rank == 0:
        try:
            img = make_image()
            s = gh.parse(img)
            tmp = path + ".part"
            img.tofile(tmp)
            os.replace(tmp, path)
            hdr = [1, s.n, s.w, s.g, s.version, int(img.size)]
            del img, s
        except Exception as ex:  # reported on every rank below
            gh_err = repr(ex)
            hdr = [0, 0, 0, 0, 0, 0]
            if dist is None:
                raise
            print(f"[rank 0] share_stream failed: {gh_err}", flush=True)
    ok, n, w, g, ver, fb = _bcast_ints(dist, hdr, device)
    if not ok:
        raise RuntimeError("rank 0 could not build the shared stream")
    return {"n": n, "w": w, "g": g, "version": ver, "file_bytes": fb}


def pick_share_dir(dist, rank: int, want_bytes: int, preferred: str, device,
                   fallbacks: Optional[List[str]] = None) -> str:
    """Directory for the shared stream file: `preferred` (normally /dev/shm, RAM-backed)
    when it has room for `want_bytes` plus 64 MiB, else the first fallback that does
    (TMPDIR, /tmp, the working directory).  Rank 0 decides (every rank of one node
    sees the same filesystems) and broadcasts its choice; raises when none fits."""
    cands = [preferred] + [d for d in (fallbacks if fallbacks is not None else
                                       [os.environ.get("TMPDIR", ""), "/tmp", os.getcwd()]) if d]
    pick = [-1]
    if rank == 0:
        for i, d in enumerate(cands):
            try:
                st = os.statvfs(d)
            except OSError:
                continue
            if os.access(d, os.W_OK) and st.f_bavail * st.f_frsize >= want_bytes + (64 << 20):
                pick = [i]
                break
    (i,) = _bcast_ints(dist, pick, device)
    if i < 0:
        raise RuntimeError(f"no directory with {want_bytes} free bytes for the shared stream: {cands}")
    return cands[i]


def exclusive_offsets(dist, count: int, device) -> Tuple[int, List[int]]:
    """Output byte offset of this rank's shard (exclusive scan of shard sizes) and
    the list of all shard sizes, via one all_gather of one integer per rank."""
    import torch

    t = torch.tensor([count], dtype=torch.int64, device=device)
    if dist is None:
        return 0, [count]
    allv = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(allv, t)
    sizes = [int(x.item()) for x in allv]
    rank = dist.get_rank()
    return sum(sizes[:rank]), sizes


def verify_slice(got: np.ndarray, seed: int, redundancy: float, offset: int,
                 threads: int = 0) -> bool:
    """Shard output == the generator's bytes [offset, offset + len(got)) (the counter-
    based generator makes any slice reproducible, so no rank needs the whole input)."""
    want = gh.generate(seed, redundancy, got.size, offset=offset, threads=threads)
    return bool(np.array_equal(got, want))


def gather_to_root(dist, shard, nbytes: int, device) -> Tuple[Optional["torch.Tensor"], float]:
    """Gather every rank's decoded shard (uint8 tensor, first `nbytes` valid) to rank 0.

    Rank 0 posts one receive per rank straight into its slice of one output buffer of
    the exact total size; the other ranks send their `nbytes` (grouped point-to-point:
    RCCL send/recv over xGMI on the GPU box).  Returns (the whole output on rank 0 /
    None elsewhere, elapsed ms of the transfer)."""
    import torch

    off, sizes = exclusive_offsets(dist, nbytes, device)
    rank, world = dist.get_rank(), dist.get_world_size()
    total = sum(sizes)
    full = torch.empty(max(1, total), dtype=torch.uint8, device=device) if rank == 0 else None
    is_cuda = device is not None and torch.device(device).type == "cuda"
    dist.barrier()
    if is_cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    if rank == 0:
        if nbytes:
            full[:nbytes].copy_(shard[:nbytes])
        ops = [dist.P2POp(dist.irecv, full[sum(sizes[:k]):sum(sizes[:k + 1])], k)
               for k in range(1, world) if sizes[k]]
    else:
        ops = [dist.P2POp(dist.isend, shard[:nbytes], 0)] if nbytes else []
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if is_cuda:
        torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    dist.barrier()
    if rank != 0:
        return None, ms
    return full[:total], ms


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


def host_threads() -> int:
    """Host threads for generate/encode: OMP_NUM_THREADS when set (16 on the GPU
    box), else the CPUs this process may run on, capped at 32."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return max(1, min(32, len(os.sched_getaffinity(0))))
    except AttributeError:  # pragma: no cover
        return max(1, min(32, os.cpu_count() or 1))
