# GPU encoder measurement: per workload, the device encode
# (bits + scan + write kernels and the gap-array memset, input resident in HBM) timed
# with HIP events, the plan step (GPU histogram + host package-merge) by wall clock,
# and the host encoder (gh_encode_write, all cores) for comparison.  Checks the image
# against the host encoder byte for byte.
# Usage: python scripts/bench_encode.py [cfg2 cfg3 cfg4]   (prints one JSON line each)
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "cse375-finalproj-huffman-decoding_amd"))
import numpy as np  # noqa: E402
import gaphuff as gh  # noqa: E402

WORKLOADS = {"cfg2": (10**8, 0.5), "cfg3": (10**9, 0.9), "cfg4": (10**9, 0.1)}
PEAK = 8000.0  # GB/s, MI355X HBM3E

for w in sys.argv[1:] or ["cfg2", "cfg3", "cfg4"]:
    n, r = WORKLOADS[w]
    data = gh.generate(375, r, n)
    with gh.Encoder(0) as e:
        e.load(data)
        t0 = time.perf_counter()
        plan = e.make_plan()
        plan_ms = (time.perf_counter() - t0) * 1e3
        for _ in range(3):
            e.encode()
        ms = sorted(e.encode() for _ in range(10))[5]
        img = e.download()
    t0 = time.perf_counter()
    host = gh.encode(data)
    host_ms = (time.perf_counter() - t0) * 1e3
    gw = (plan.g + 7) // 8
    alg = n + 4 * plan.w + 4 * gw  # input read once, payload + gaps written once
    print(json.dumps({
        "workload": w, "n": n, "redundancy": r, "encode_ms": round(ms, 4),
        "input_GBps": round(n / ms / 1e6, 1), "alg_bytes": alg,
        "roofline_frac": round(alg / ms / 1e6 / PEAK, 3),
        "plan_ms_wall": round(plan_ms, 2), "host_encode_ms_wall": round(host_ms, 1),
        "host_threads": os.cpu_count(), "identical_to_host": bool(np.array_equal(img, host)),
    }), flush=True)
