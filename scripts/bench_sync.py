# Self-synchronising decode measurement: per workload, the raw
# (gap-less) stream = the gap-array image's payload.  Times gh_sync_gaps (walk kernel +
# first verify pass, HIP events; input resident in HBM) and the gap-array decode of the
# stream loaded through gh_ctx_load_raw; checks the synthesised gap words against the
# encoder's and the decoded bytes against the input.
# Usage: python scripts/bench_sync.py [--halo H] [cfg2 cfg3 cfg4]   (prints one JSON line each;
# --halo forces the warm-up segments per lane, GH_SYNC_HALO, e.g. 0 for many repairs)
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "cse375-finalproj-huffman-decoding_amd"))
import numpy as np  # noqa: E402
import gaphuff as gh  # noqa: E402

WORKLOADS = {"cfg2": (10**8, 0.5), "cfg3": (10**9, 0.9), "cfg4": (10**9, 0.1)}
PEAK = 8000.0  # GB/s, MI355X HBM3E


def arr(ptr, n):
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint32)), (max(n, 1),))[:n]


args = sys.argv[1:]
forced = None
if args[:1] == ["--halo"]:
    forced = args[1]
    os.environ["GH_SYNC_HALO"] = forced
    args = args[2:]
for wl in args or ["cfg2", "cfg3", "cfg4"]:
    n, r = WORKLOADS[wl]
    data = gh.generate(375, r, n)
    s = gh.parse(gh.encode(data, threads=16))
    syms = s.symbols
    payload = arr(s.c.payload, s.w).copy()
    gw = (s.g + 7) // 8
    want_gaps = arr(s.c.gap_words, gw).copy()
    with gh.DeviceBuffer(4 * (s.w + 16)) as dw, gh.DeviceBuffer(4 * (gw + 4)) as dg:
        dw.upload(payload)
        for _ in range(3):
            gh.sync_gaps(syms, dw.addr, s.w, dg.addr)
        reps = [gh.sync_gaps(syms, dw.addr, s.w, dg.addr) for _ in range(10)]
        sync_ms = float(np.median([x.kernel_ms for x in reps]))
        host_ms = float(np.median([x.host_ms for x in reps]))  # the halo estimate (not in kernel_ms)
        got = dg.download(np.empty(gw, np.uint32))
    with gh.Decoder(0) as d:
        rep0 = d.load_raw(syms, n, payload)
        for _ in range(3):
            d.decode(timed=False)
        d.report()
        d.reset_timing()
        for _ in range(10):
            d.decode()
        rep = d.report()
        out = d.download(n)
    alg_sync = 4 * s.w + 4 * gw  # payload read once, gap words written once
    alg_dec = 4 * s.w + 4 * gw + n
    total = sync_ms + rep.kernel_ms
    print(json.dumps({
        "workload": wl, "n": n, "redundancy": r, "w": s.w, "g": s.g, "halo_forced": forced is not None,
        "sync_ms": round(sync_ms, 4), "sync_roofline_frac": round(alg_sync / sync_ms / 1e6 / PEAK, 3),
        "sync_host_ms": round(host_ms, 4), "sync_call_ms": round(sync_ms + host_ms, 4), "halo": int(reps[-1].halo),
        "sync_alg_bytes": alg_sync, "mismatches": int(reps[-1].mismatches), "passes": int(reps[-1].passes),
        "decode_ms": round(rep.kernel_ms, 4), "decode_mode": gh.MODE_NAMES.get(rep.mode),
        "decode_path": gh.PATH_NAMES.get(rep.path),
        "raw_total_ms": round(total, 4), "raw_decoded_GBps": round(n / total / 1e6, 1),
        "raw_roofline_frac": round(alg_dec / total / 1e6 / PEAK, 3),
        "gaps_identical": bool(np.array_equal(got, want_gaps)), "load_mismatches": int(rep0.mismatches),
        "bitexact": bool(np.array_equal(out, data)),
    }), flush=True)
