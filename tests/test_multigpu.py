"""N>1 path on CPU: gap-segment sharding, shard offsets, gather to rank 0 (gloo).

Rank 0 builds the global stream once and shares it as a file (gh_dist.share_stream,
as bench.py does under /dev/shm); each rank takes its shard from
gh_dist.shard_range, checks it against the generator's slice at its output offset
(gh_dist.verify_slice), and stands in for the GPU shard decode with the CPU oracle
(bit-serial decode of the stream, sliced at the shard's segment-count offsets) —
the oracle is the checker here, not the thing measured.  The collectives are the
ones bench.py runs over RCCL on the GPU box (gh_dist)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, r, path, q):
    import sys
    for p in (os.path.join(ROOT, "cse375-finalproj-huffman-decoding_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import gaphuff as gh
    import gh_dist
    import oracle

    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        # rank 0 builds the global stream once; the others only learn its header
        hdr = gh_dist.share_stream(dist, rank, path,
                                   lambda: gh.encode(gh.generate(375, r, n), threads=2), "cpu")
        assert hdr["n"] == n
        b, e = gh_dist.shard_range(hdr["g"], world, rank)
        img = np.fromfile(path, dtype=np.uint8)
        assert img.size == hdr["file_bytes"]
        counts = [oracle.segment_count(img, i) for i in range(hdr["g"])]
        full, _ = oracle.decode(img)
        # the last segment may decode tail padding bits: outputs clamp at N
        lo, hi = min(sum(counts[:b]), n), min(sum(counts[:e]), n)
        shard = torch.from_numpy(full[lo:hi].copy())
        off, sizes = gh_dist.exclusive_offsets(dist, hi - lo, "cpu")
        assert off == lo, (off, lo)
        assert sum(sizes) == n
        assert gh_dist.verify_slice(shard.numpy(), 375, r, off)
        if hi > lo:  # a corrupted shard must fail its slice check
            bad = shard.numpy().copy()
            bad[-1] ^= 1
            assert not gh_dist.verify_slice(bad, 375, r, off)
        mx, sm = gh_dist.reduce_max_sum(dist, [float(rank), float(hi - lo)], "cpu")
        assert mx[0] == world - 1 and sm[1] == n
        out, ms = gh_dist.gather_to_root(dist, shard, hi - lo, "cpu")
        ok = True
        if rank == 0:
            ok = out is not None and np.array_equal(out.numpy(), gh.generate(375, r, n))
        else:
            ok = out is None
        ok = gh_dist.all_true(dist, ok, "cpu")
        q.put((rank, ok, b, e, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # pragma: no cover - reported to the parent
        q.put((rank, False, -1, -1, repr(ex)))


@pytest.mark.parametrize("world,n,r", [(2, 40000, 0.5), (3, 25000, 0.1), (2, 5, 0.9), (4, 3000, 0.5)])
def test_sharded_gather_gloo(world, n, r, tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    path = str(tmp_path / "shared.huff")
    procs = [ctx.Process(target=_worker, args=(k, world, port, n, r, path, q)) for k in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    res.sort()
    assert all(x[4] is None for x in res), res
    assert all(x[1] for x in res), res
    # shards tile the segment range
    assert res[0][2] == 0
    for a, c in zip(res, res[1:]):
        assert a[3] == c[2]


def test_shard_alg_bytes():
    import gh_dist
    # whole stream: payload W words (+0 extra: 4e+1 clamps to W), ceil(G/8) gap words, N out
    assert gh_dist.shard_alg_bytes(w=40, begin=0, end=10, out_bytes=100) == 4 * 40 + 4 * 2 + 100
    # interior shard reads one word past its last segment (spanning codeword)
    assert gh_dist.shard_alg_bytes(w=400, begin=8, end=16, out_bytes=7) == 4 * 33 + 4 * 1 + 7


def _pick_worker(rank, world, port, dirs, want, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "cse375-finalproj-huffman-decoding_amd"))
    import torch.distributed as dist

    import gh_dist

    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        try:
            got = gh_dist.pick_share_dir(dist, rank, want, dirs[0], "cpu", fallbacks=dirs[1:])
        except RuntimeError:
            got = None
        q.put((rank, got, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # pragma: no cover - reported to the parent
        q.put((rank, None, repr(ex)))


@pytest.mark.parametrize("case", ["fits", "fallback", "none"])
def test_share_dir_free_space_gloo(case, tmp_path):
    """bench.py's shared stream file: rank 0 checks the preferred directory's free space
    (os.statvfs) and falls back to the next directory that has room; every rank gets the
    same answer (a broadcast), and no room anywhere is an error on every rank."""
    free = os.statvfs(str(tmp_path)).f_bavail * os.statvfs(str(tmp_path)).f_frsize
    missing = str(tmp_path / "does_not_exist")
    dirs = {"fits": [str(tmp_path), missing], "fallback": [missing, str(tmp_path)],
            "none": [missing, missing]}[case]
    want = 1 << 20 if case != "none" else free * 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pick_worker, args=(k, 2, port, dirs, want, q)) for k in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert all(x[2] is None for x in res), res
    expect = None if case == "none" else str(tmp_path)
    assert [x[1] for x in res] == [expect, expect]
