#!/usr/bin/env python3
"""bench.py — decoded GB/s of the gap-array Huffman decode hot path on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is
launched by ``torch.distributed.run`` (one rank per GPU, RCCL).  Rank 0 prints ONE
JSON line on stdout; everything else goes to stderr.

Workload (BASELINE.json ``configs``): a "step" is one decode of one resident
compressed.huff shard — the gap-array prescan + per-segment table decode done by
the HIP kernels behind ``gh_ctx_decode`` (include/gaphuff.h).  Default ``cfg4`` =
configs[3]: 10^9 bytes of generate.cpp-distributed data, redundancy 0.1, per GPU
(compressed payload 1.01 GB: the north star's "1 GB compressed.huff"; it does not fit
the 256 MiB Infinity Cache, so every decode streams from HBM).  ``--workload
cfg2|cfg3|cfg5`` selects the others.  The same run then times a second workload (``--sub``,
default ``cfg5``: redundancy 0.5, 1 GB per GPU, so 8 GB over 8 GPUs = configs[4] literally,
with its own bit-exact check and RCCL gather) and reports it under ``sub``; ``--sub none``
skips it.

Weak scaling: at N GPUs the global input is N x 10^9 bytes.  Rank 0 generates and
encodes the global stream ONCE (v2 header when N, W or G >= 2^31) into a file under
/dev/shm; every rank streams only its own shard of gap segments (``gh_plan_shards``)
from that file to its GPU (``gh_ctx_load_file``) — no data-path collective.  After
the timed region each rank checks its decoded shard byte-for-byte against the
generator's slice at the shard's output offset (exclusive scan of the shard sizes),
and the shards are gathered to rank 0 over RCCL send/recv (timed separately,
``gather_ms``) and checked again there.

``value`` = decoded bytes of all ranks per step x K / max-over-ranks wall time of the
K steps (inputs resident in HBM).  ``roofline.achieved`` = algorithmic bytes per
decode (compressed payload + gap words + decoded output) / the
decode's average duration, measured with HIP events recorded by the library on the
stream the kernels are launched on (torch's current stream).  ``roofline.copy_frac``
= achieved / the rate of a streaming copy (gh_bw_copy) moving the same bytes on the
same GPU.  ``cpu_baseline`` times the reference's own CPU programs (compiled from
their sources into oracle/_ref by oracle/Makefile) on a bounded sample, rank 0 at
N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "cse375-finalproj-huffman-decoding_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

import gaphuff as gh  # noqa: E402
import gh_dist  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)

WORKLOADS = {
    # name: (bytes per GPU, redundancy, description)
    "cfg2": (10**8, 0.5, "configs[1]: 100 MB generate.cpp data, redundancy=0.5, per GPU"),
    "cfg3": (10**9, 0.9, "configs[2]: 1 GB, redundancy=0.9 (short codes), per GPU"),
    "cfg4": (10**9, 0.1, "configs[3]: 1 GB, redundancy=0.1 (1.01 GB compressed), per GPU"),
    "cfg5": (10**9, 0.5, "configs[4]: 1 GB per GPU (8 GB at 8 GPUs), redundancy=0.5"),
}


# (mode, path) -> the kernels one decode launches (rocprofv3 names); path -1 = any
KERNEL_NAMES = {
    (1, 4): "gh::gh_ws_count_kernel + gh::gh_ws_scan_kernel + gh::gh_ws_write_kernel",
    (2, -1): "gh::gh_tile_kernel",
    (4, -1): "gh::gh_mtile_kernel",
}


# How gh_ctx_decode times a decode (kernel_ms), per mode: the tile kernels take their start
# and stop timestamps in the dispatch packet itself (hipExtLaunchKernel); the wave split
# records HIP marker events around its three kernels (the markers sit inside the interval).
KERNEL_TIMING = {
    1: "HIP events around the count, scan and write kernels",
    2: "dispatch-packet timestamps (hipExtLaunchKernel start/stop events)",
    4: "dispatch-packet timestamps (hipExtLaunchKernel start/stop events)",
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(r: float, seed: int, sample: int) -> dict:
    """The reference's CPU decoders on a bounded sample (rank 0, N=1 only).

    The oracle module is test infrastructure: here it is only the timing harness for
    the reference binaries built from the reference's own sources (oracle/_ref)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (checker / baseline only)

    data = gh.generate(seed, r, sample)
    nproc = os.cpu_count() or 1
    extra = []
    if oracle.ref_available("sequential"):
        res = oracle.run_reference_cpu("sequential", data)
        base = {
            "value": round(sample / (res["decode_us"] * 1e-6) / 1e9, 6), "unit": "GB/s",
            "cores": 1, "kind": "reference",
            "sample": (f"{sample} B generate(r={r}, seed={seed}) (the bench workload's redundancy); "
                       f"reference sequential.cpp decode() timed by its own clock: "
                       f"{res['decode_us'] / 1e6:.3f} s, verification {'PASS' if res['verified'] else 'FAIL'}"),
        }
        runs = [("parallel_cpu_prescan", None), ("parallel_cpu_prescan", nproc),
                ("parallel_decomp_cpu", None), ("parallel_decomp_cpu", nproc)]
        for name, thr in runs:
            if not oracle.ref_available(name if thr is None else
                                        {"parallel_cpu_prescan": "prescan_driver",
                                         "parallel_decomp_cpu": "decomp_driver"}[name]):
                continue
            try:
                o = oracle.run_reference_cpu(name, data, timeout=120 if thr is None else 90, threads=thr)
                extra.append({"program": name, "threads": o["threads"],
                              "threads_source": "as shipped" if thr is None else "nproc",
                              "value": round(sample / (o["decode_us"] * 1e-6) / 1e9, 6),
                              "unit": "GB/s", "verified": o["verified"]})
            except Exception as e:  # reported, not fatal
                extra.append({"program": name, "threads": thr, "error": str(e)[:200]})
    else:
        # Restated port (oracle/gh_oracle.c, bit-serial) when oracle/_ref was not built.
        img = oracle.encode(data)
        t0 = time.perf_counter()
        dec, _ = oracle.decode(img)
        dt = time.perf_counter() - t0
        base = {"value": round(sample / dt / 1e9, 6), "unit": "GB/s", "cores": 1, "kind": "port",
                "sample": f"{sample} B generate(r={r}, seed={seed}); oracle bit-serial decode, "
                          f"{dt:.3f} s, verified {bool(np.array_equal(dec, data))}"}
    if oracle.ref_available("sequential"):
        # BASELINE configs[0] literally: sequential.cpp on 10 MB of redundancy-0.5 data
        try:
            d1 = gh.generate(seed, 0.5, 10**7)
            o = oracle.run_reference_cpu("sequential", d1)
            extra.append({"program": "sequential", "config": "configs[0]: 10^7 B, redundancy 0.5",
                          "threads": 1, "value": round(10**7 / (o["decode_us"] * 1e-6) / 1e9, 6),
                          "unit": "GB/s", "decode_s": round(o["decode_us"] / 1e6, 4),
                          "verified": o["verified"]})
        except Exception as e:  # reported, not fatal
            extra.append({"program": "sequential", "config": "configs[0]", "error": str(e)[:200]})
    if extra:
        base["others"] = extra
    base["host_cpus"] = nproc
    base["omp_num_threads_env"] = os.environ.get("OMP_NUM_THREADS")
    try:
        with open("/proc/cpuinfo") as f:
            base["cpu_model"] = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        pass
    return base


def load_traffic(workload: str, per_gpu: int, n_gpus: int):
    """PMC-derived HBM bytes per launch from the committed rocprofv3 counter summary,
    keyed by (workload, bytes per GPU, GPUs); None when no pass matches exactly."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
        e = t.get(f"{workload}_{per_gpu}_n{n_gpus}")
        if e is None:
            return None, None
        # the source names the kernel(s) the counters were read from first
        return float(e["bytes_per_launch"]), f"{' + '.join(e.get('kernels', []))} (round {e.get('round')}): {e.get('source')}"
    except (OSError, ValueError, KeyError):
        return None, None


def copy_yardstick(nbytes: int, stream: int, device) -> float:
    """GB/s (bytes read + written) of gh_bw_copy moving `nbytes` in total."""
    import torch

    half = max(16, (nbytes // 2) & ~15)
    src = torch.empty(half, dtype=torch.uint8, device=device)
    dst = torch.empty(half, dtype=torch.uint8, device=device)
    src.fill_(7)
    ms = gh.bw_copy(dst.data_ptr(), src.data_ptr(), half, stream, reps=10)
    del src, dst
    return 2 * half / (ms * 1e-3) / 1e9


def end_to_end(img: np.ndarray, args, r: float, dev, threads: int) -> dict:
    """File in, file out, never part of `value`: the compressed image is written to a
    file (untimed), then timed: a fresh context streams it to HBM (gh_ctx_load_file),
    decodes it and streams the output to a second file (gh_ctx_save_file).  Also timed
    in the reference's own scope (decoder/src/huff.cpp:106-129: host buffer -> device,
    decode, device -> host buffer; file reads and fwrite outside it).  The output file
    is checked against the generator."""
    import torch

    s = gh.parse(img)
    n = s.n
    d = gh_dist.pick_share_dir(None, 0, int(img.size) + n, args.shm, dev)
    src = os.path.join(d, f"gh_e2e_{os.getpid()}.huff")
    dst = os.path.join(d, f"gh_e2e_{os.getpid()}.out")
    res = {"dir": d}
    try:
        img.tofile(src)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with gh.Decoder(dev.index or 0) as d2:
            d2.load_file(src)
            t1 = time.perf_counter()
            d2.decode()
            rep = d2.report()
            t2 = time.perf_counter()
            d2.save_file(dst, n)
            t3 = time.perf_counter()
        res.update({"file_to_file_ms": round((t3 - t0) * 1e3, 2), "load_file_ms": round((t1 - t0) * 1e3, 2),
                    "decode_ms": round((t2 - t1) * 1e3, 3), "save_file_ms": round((t3 - t2) * 1e3, 2),
                    "file_to_file_gbps": round(n / (t3 - t0) / 1e9, 3), "status": int(rep.status)})
        out = np.memmap(dst, dtype=np.uint8, mode="r")
        ok = out.size == n
        step = 1 << 27
        for off in range(0, n, step):
            if not ok:
                break
            ok = gh_dist.verify_slice(np.asarray(out[off:off + step]), args.seed, r, off, threads=threads)
        del out
        res["bitexact"] = bool(ok)
        # the reference's scope: host image -> HBM, decode, HBM -> host buffer
        host = np.empty(n, dtype=np.uint8)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with gh.Decoder(dev.index or 0) as d3:
            d3.load(s)
            d3.decode()
            d3.report()
            host[:] = d3.download(n)
        res["ref_scope_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
        res["ref_scope_note"] = ("decoder_l1_l2 scope: context + H2D (pageable) + decode + D2H, "
                                 "as the reference's 'Decode time' (huff.cpp:106-129)")
        del host, s
    finally:
        for f in (src, dst):
            try:
                os.unlink(f)
            except OSError:
                pass
    return res


def run_workload(args, name: str, per_gpu: int, r: float, ctx: dict, keep_image: bool) -> dict:
    """One timed workload: build (or share) the stream, load this rank's shard, W untimed
    and K timed decodes between barriers, then the correctness checks and the RCCL
    gather.  Returns the measurements (rank-local values plus max/sum over ranks)."""
    import torch

    world, rank, dev, dist, use_dist, threads = (ctx[k] for k in ("world", "rank", "dev", "dist", "use_dist",
                                                                   "threads"))
    total = per_gpu * world
    t0 = time.time()
    dec = gh.Decoder(ctx["local"])
    res = {"image": None, "share_dir": None}
    try:
        if not use_dist:
            data = gh.generate(args.seed, r, total, threads=threads)
            img = gh.encode(data, threads=threads)
            del data
            s = gh.parse(img)
            hdr = {"n": s.n, "w": s.w, "g": s.g, "version": s.version, "file_bytes": int(img.size)}
            b, e = 0, s.g
            t1 = time.time()
            dec.load(s)
            torch.cuda.synchronize()
            load_ms = (time.time() - t1) * 1e3
            del s
            if keep_image:
                res["image"] = img
            del img
        else:
            port = os.environ.get("MASTER_PORT", "0")
            # the stream file: about the input size (r >= 0 codes average <= 8.1 bits a byte)
            share_dir = gh_dist.pick_share_dir(dist, rank, int(total * 1.05) + (1 << 20), args.shm, dev)
            res["share_dir"] = share_dir
            path = os.path.join(share_dir, f"gh_bench_{port}_{name}_{per_gpu}_{world}.huff")
            if rank == 0 and share_dir != args.shm:
                log(f"[rank 0] {args.shm} lacks room for the stream: using {share_dir}")

            def make_image():
                d = gh.generate(args.seed, r, total, threads=threads)
                return gh.encode(d, threads=threads)

            try:
                hdr = gh_dist.share_stream(dist, rank, path, make_image, dev)
                b, e = gh_dist.shard_range(hdr["g"], world, rank)
                t1 = time.time()
                dec.load_file(path, b, e)
                torch.cuda.synchronize()
                load_ms = (time.time() - t1) * 1e3
                dist.barrier()
            finally:  # never leave the stream in RAM-backed tmpfs, whatever failed
                if rank == 0:
                    for f in (path, path + ".part"):
                        try:
                            os.unlink(f)
                        except OSError:
                            pass
        log(f"[rank {rank}] {name}: N={hdr['n']} W={hdr['w']} G={hdr['g']} v{hdr['version']} shard=[{b},{e}) "
            f"setup {t1 - t0:.1f}s load {load_ms:.1f} ms")

        stream = torch.cuda.current_stream().cuda_stream
        # decodes go on the decoder's own stream (0): back-to-back tile decodes there need no
        # device-chain wait packet (gh_ctx_decode); the timed region is bracketed by device-
        # wide synchronisations, and copy_output waits for the last decode on torch's stream
        dstream = 0
        for _ in range(args.warmup):
            dec.decode(dstream, timed=False)
        rep0 = dec.report(dstream)  # synchronises, checks status of the warmup launches
        dec.reset_timing()

        def barrier():
            if dist is not None:
                dist.barrier()

        barrier()
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for _ in range(args.steps):
            dec.decode(dstream, timed=True)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - ts
        barrier()
        rep = dec.report(dstream)
        shard_bytes = int(rep.out_bytes)
        # Sustained rate, untimed by the contract and reported beside it: the kernel time of
        # a GPU that has just come out of idle dips for ~40 launches (the clock settles under
        # the new load: per-dispatch 456 -> 615 -> 430 us on cfg4, profiles/r05_burst_series.txt),
        # and K = 20 after W = 5 sits in that dip.  S more back-to-back decodes, the mean of
        # all and of the second half.
        sustained = None
        if args.sustain > 0:
            halves = []
            for part in (args.sustain // 2, args.sustain - args.sustain // 2):
                dec.reset_timing()
                for _ in range(part):
                    dec.decode(dstream, timed=True)
                halves.append(float(dec.report(dstream).kernel_ms))
            sustained = {"launches": args.sustain, "kernel_ms_mean": round(sum(halves) / 2, 4),
                         "kernel_ms_second_half": round(halves[1], 4)}

        alg = gh_dist.shard_alg_bytes(hdr["w"], b, e, shard_bytes)
        kern_ms = float(rep.kernel_ms)
        mx, sm = gh_dist.reduce_max_sum(dist, [elapsed, kern_ms, float(shard_bytes)], dev)

        # ---- correctness: each shard vs the generator's slice at its output offset
        off, sizes = gh_dist.exclusive_offsets(dist, shard_bytes, dev)
        out = torch.empty(max(1, shard_bytes), dtype=torch.uint8, device=dev)
        dec.copy_output(out.data_ptr(), shard_bytes, 0, stream)
        torch.cuda.synchronize()
        ok = (sum(sizes) == hdr["n"]) and gh_dist.verify_slice(out[:shard_bytes].cpu().numpy(), args.seed, r, off,
                                                               threads=threads)
        status_ok = rep.status == 0 and rep0.status == 0
        gather_ms = None
        gather_ok = None
        if dist is not None and not args.no_gather:
            full, gather_ms = gh_dist.gather_to_root(dist, out, shard_bytes, dev)
            if rank == 0:
                gather_ok = full is not None and full.numel() == hdr["n"]
                for k in range(world):  # gathered shard k == generator slice, compared on the GPU
                    if not gather_ok:
                        break
                    lo = sum(sizes[:k])
                    want = torch.from_numpy(gh.generate(args.seed, r, sizes[k], offset=lo, threads=threads)).to(dev)
                    gather_ok = bool(torch.equal(full[lo:lo + sizes[k]], want))
                    del want
                del full
            ok = ok and (gather_ok is not False)
        ok = gh_dist.all_true(dist, bool(ok and status_ok), dev)
        del out
        torch.cuda.empty_cache()
        res.update({"hdr": hdr, "b": b, "e": e, "rep": rep, "alg": alg, "kern_ms": kern_ms,
                    "max_elapsed": mx[0], "max_kern": mx[1], "sum_bytes": sm[2], "ok": ok,
                    "gather_ms": gather_ms, "gather_ok": gather_ok, "load_ms": load_ms, "total": total,
                    "sustained": sustained})
        return res
    finally:
        dec.close()


def sustained_record(res: dict):
    """The 'sustained' key: kernel time over S more back-to-back decodes (this rank's), as
    a roofline fraction too (same algorithmic bytes).  Not the contract's value."""
    su = res.get("sustained")
    if not su:
        return None
    out = dict(su)
    for k in ("kernel_ms_mean", "kernel_ms_second_half"):
        if su[k] > 0:
            out[k.replace("kernel_ms", "roofline_frac")] = round(res["alg"] / (su[k] * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
    out["note"] = ("untimed by the contract: the clock settles during the first ~40 launches after idle "
                   "(profiles/r05_burst_series.txt); K steps after W warmups measure that transient")
    return out


def sub_record(args, name: str, res: dict, r: float, desc: str, per_gpu: int) -> dict:
    """A second workload timed in the same run (rank 0's summary of run_workload)."""
    kern_ms = res["kern_ms"]
    achieved = res["alg"] / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    rep = res["rep"]
    return {"workload": name, "description": desc, "bytes_per_gpu": per_gpu, "global_bytes": res["total"],
            "redundancy": r, "compressed_bytes": res["hdr"]["file_bytes"], "segments": res["hdr"]["g"],
            "format_version": res["hdr"]["version"],
            "value": round(res["sum_bytes"] * args.steps / res["max_elapsed"] / 1e9, 3), "unit": "GB/s",
            "ms_per_step": round(res["max_elapsed"] / args.steps * 1e3, 4),
            "kernel_ms": round(kern_ms, 4), "max_kernel_ms_over_ranks": round(res["max_kern"], 4),
            "roofline_frac": round(achieved / HBM_PEAK_GBPS, 4), "alg_bytes_per_launch": res["alg"],
            "mode": gh.MODE_NAMES.get(int(rep.mode)), "path": gh.PATH_NAMES.get(int(rep.path)),
            "bitexact": bool(res["ok"]),
            "gather_ms": None if res["gather_ms"] is None else round(res["gather_ms"], 3),
            "gather_bitexact": res["gather_ok"], "load_ms": round(res["load_ms"], 2),
            "sustained": sustained_record(res)}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--sustain", type=int, default=200,
                    help="after the timed steps: this many more decodes, reported as 'sustained' (0: skip)")
    ap.add_argument("--workload", default="cfg4", choices=sorted(WORKLOADS))
    ap.add_argument("--sub", default="cfg5", choices=sorted(WORKLOADS) + ["none"],
                    help="second workload timed in the same run, reported under 'sub' (default cfg5: "
                         "r=0.5, 1 GB per GPU = configs[4] at 8 GPUs, with its own RCCL gather)")
    ap.add_argument("--size", type=int, default=0, help="bytes per GPU (overrides workload and sub)")
    ap.add_argument("--seed", type=int, default=375)
    ap.add_argument("--cpu-sample", type=int, default=10**8,
                    help="bytes decoded by the CPU baseline (0 = skip)")
    ap.add_argument("--threads", type=int, default=0, help="host threads for generate/encode (0 = auto)")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the RCCL output gather")
    ap.add_argument("--no-copy", action="store_true", help="skip the streaming-copy yardstick")
    ap.add_argument("--shm", default="/dev/shm", help="N>1: directory of the shared stream file "
                    "(checked for free space; falls back to TMPDIR, /tmp or the working directory)")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the multi-GPU path (torch.distributed over RCCL, shared stream file, "
                         "per-rank file loading, offsets, RCCL gather) even at one rank")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end file-to-file timing")
    ap.add_argument("--out-json", default="", help="also write the JSON line to this file (rank 0)")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    use_dist = world > 1 or args.force_dist
    if use_dist:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=dev)
    threads = args.threads or gh_dist.host_threads()
    ctx = {"world": world, "rank": rank, "local": local, "dev": dev, "dist": dist, "use_dist": use_dist,
           "threads": threads}

    per_gpu, r, desc = WORKLOADS[args.workload]
    if args.size:
        per_gpu = args.size
    res = run_workload(args, args.workload, per_gpu, r, ctx, keep_image=not use_dist and not args.no_e2e)
    e2e_img = res.pop("image")
    rep, alg, kern_ms = res["rep"], res["alg"], res["kern_ms"]
    hdr, shard_bytes = res["hdr"], int(res["rep"].out_bytes)
    ok = res["ok"]

    stream = torch.cuda.current_stream().cuda_stream
    copy_gbps = None
    if rank == 0 and not args.no_copy:
        try:
            copy_gbps = copy_yardstick(alg, stream, dev)
        except Exception as ex:  # the yardstick must not hide the decode number
            log(f"copy yardstick failed: {ex}")

    e2e = None
    if e2e_img is not None:
        try:
            e2e = end_to_end(e2e_img, args, r, dev, threads)
        except Exception as ex:  # reported, never hides the decode number
            e2e = {"error": str(ex)[:300]}
        del e2e_img

    # the second workload (default configs[4]'s r=0.5 stream: 1 GB per GPU, RCCL gather)
    sub = None
    if args.sub != "none" and args.sub != args.workload:
        s_per_gpu, s_r, s_desc = WORKLOADS[args.sub]
        if args.size:
            s_per_gpu = args.size
        try:
            sres = run_workload(args, args.sub, s_per_gpu, s_r, ctx, keep_image=False)
            if rank == 0:
                sub = sub_record(args, args.sub, sres, s_r, s_desc, s_per_gpu)
            ok = ok and sres["ok"]
        except Exception as ex:  # reported; a failed sub-record fails the run
            log(f"[rank {rank}] sub-workload {args.sub} failed: {ex}")
            sub = {"workload": args.sub, "error": str(ex)[:300], "bitexact": False}
            ok = False
        ok = gh_dist.all_true(dist, bool(ok), dev)

    if rank == 0:
        achieved = alg / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
        read_bytes = alg - shard_bytes
        traffic, tsrc = load_traffic(args.workload, per_gpu, world)
        line = {
            "metric": "decoded GB/s",
            "value": round(res["sum_bytes"] * args.steps / res["max_elapsed"] / 1e9, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(res["max_elapsed"] / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic: seeded generate.cpp distribution (redundancy {r}), encoded by the "
                    f"in-repo gap-array encoder (reference boundary_PM code lengths)",
            "config": {"workload": args.workload, "description": desc, "bytes_per_gpu": per_gpu,
                       "global_bytes": res["total"], "redundancy": r, "compressed_bytes": hdr["file_bytes"],
                       "format_version": hdr["version"], "segments": hdr["g"],
                       "parallelism": f"gap-segment shards x{world}",
                       "lut_bits": int(rep.lut_bits), "grid": int(rep.grid)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic,
                         "copy_gbps": None if copy_gbps is None else round(copy_gbps, 1),
                         "copy_frac": None if not copy_gbps else round(achieved / copy_gbps, 4),
                         "read_frac": round(read_bytes / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
                         if kern_ms > 0 else None,
                         "kernel": KERNEL_NAMES.get((int(rep.mode), int(rep.path)),
                                                    KERNEL_NAMES.get((int(rep.mode), -1))),
                         "mode": gh.MODE_NAMES.get(int(rep.mode)),
                         "path": gh.PATH_NAMES.get(int(rep.path)),
                         "kernel_ms": round(kern_ms, 4), "max_kernel_ms_over_ranks": round(res["max_kern"], 4),
                         "alg_bytes_per_launch": alg,
                         "traffic_source": tsrc,
                         "kernel_timing": KERNEL_TIMING.get(int(rep.mode))},
            "bitexact": bool(res["ok"]),
            "gather_ms": None if res["gather_ms"] is None else round(res["gather_ms"], 3),
            "gather_bitexact": res["gather_ok"],
            "load_ms": round(res["load_ms"], 2),
            "load_kind": (("host memory -> HBM (pageable)" if os.environ.get("GH_H2D") == "pageable"
                           or res.get("load_bytes", 1 << 30) < (8 << 20) else
                           "host memory -> pinned double-buffered staging -> HBM (the first load "
                           "of a process also pins the staging set)") if not use_dist else
                         f"gh_ctx_load_file: {res['share_dir']} file -> pinned -> HBM, shard words only"),
            "dist": {"backend": "nccl (RCCL)", "world": world, "forced": bool(args.force_dist and world == 1),
                     "share_dir": res["share_dir"]} if use_dist else None,
            "e2e": e2e,
            "sustained": sustained_record(res),
            "sub": sub,
        }
        if world == 1 and not use_dist and args.cpu_sample > 0:
            try:
                line["cpu_baseline"] = cpu_baseline(r, args.seed, args.cpu_sample)
            except Exception as ex:  # a missing baseline must not hide the GPU number
                line["cpu_baseline"] = {"value": None, "unit": "GB/s", "cores": 1, "kind": "reference",
                                        "sample": f"failed: {ex}"[:300]}
        print(json.dumps(line), flush=True)
        if args.out_json:
            with open(args.out_json, "w") as f:
                f.write(json.dumps(line) + "\n")
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
