# Timing of the decode structures the launcher uses for codes the tile kernel and the
# wave split do not take (codes > 12 bits or minlen 1): streams whose code lengths reach
# 16 bits, 10^8 and 10^9 bytes.  Prints one line per stream: path, kernel time, the
# fraction of the 8 TB/s HBM peak on algorithmic bytes, bit-exactness.
# Usage: python scripts/time_longcodes.py [--n 100000000,1000000000] [--q 0.5,0.7]
import argparse, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cse375-finalproj-huffman-decoding_amd"))
import numpy as np, gaphuff as gh
ap = argparse.ArgumentParser()
ap.add_argument("--n", default="100000000,1000000000")
ap.add_argument("--q", default="0.5,0.7")
a = ap.parse_args()
rng = np.random.default_rng(7)
for n in [int(x) for x in a.n.split(",")]:
    for q in [float(x) for x in a.q.split(",")]:
        name = f"geometric_q{q}"
        p = q ** np.arange(256, dtype=np.float64)
        p /= p.sum()
        data = rng.choice(256, size=n, p=p).astype(np.uint8)
        img = gh.encode(data, threads=16)
        s = gh.parse(img)
        lens = [l for _, l in s.symbols]
        d = gh.Decoder(0); d.load(s)
        for _ in range(3): d.decode(timed=False)
        d.report(); d.reset_timing()
        for _ in range(10): d.decode()
        rep = d.report()
        alg = 4 * s.w + 4 * ((s.g + 7) // 8) + s.n
        ok = bool(np.array_equal(d.download(s.n), data)) and rep.status == 0
        print(f"{name} n={n} minlen={min(lens)} maxlen={max(lens)} mode={gh.MODE_NAMES.get(rep.mode)} "
              f"path={gh.PATH_NAMES.get(rep.path)} ms={rep.kernel_ms:.4f} frac={alg / rep.kernel_ms / 1e6 / 8000:.4f} "
              f"GB/s={n / rep.kernel_ms / 1e6:.1f} ok={ok}", flush=True)
        d.close()
