# One workload, one lib (GAPHUFF_LIB): QO_WARM (default 3) untimed decodes, then `reps`
# timed; prints the average kernel time, roofline fraction and bit-exactness.  (A GPU
# out of idle runs its first ~40 decodes at a lower clock: QO_WARM=60 with 100 reps
# times the steady state, the low-noise A/B setting.)
# Usage: python scripts/quick_one.py name:N:r [reps]   (name geo*: r is a geometric q)
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'cse375-finalproj-huffman-decoding_amd'))
import numpy as np, gaphuff as gh
name, n, r = sys.argv[1].split(":"); n = int(n); r = float(r)
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
if name.startswith("geo"):  # geo*:N:q — geometric byte distribution p_i ~ q^i (long codes, time_longcodes.py)
    p = r ** np.arange(256, dtype=np.float64)
    data = np.random.default_rng(7).choice(256, size=n, p=p / p.sum()).astype(np.uint8)
else:
    data = gh.generate(375, r, n)
img = gh.encode(data); s = gh.parse(img)
alg = 4 * s.w + 4 * ((s.g + 7) // 8) + s.n
d = gh.Decoder(0); d.load(s)
for _ in range(int(os.environ.get('QO_WARM', '3'))): d.decode(timed=False)
d.report(); d.reset_timing()
for _ in range(reps): d.decode()
rep = d.report()
ok = bool(np.array_equal(d.download(s.n), data)) and rep.status == 0
print(f"{name} ms={rep.kernel_ms:.4f} frac={alg / rep.kernel_ms / 1e6 / 8000:.4f} mode={gh.MODE_NAMES.get(rep.mode)} "
      f"K={rep.lut_bits} grid={rep.grid} st={rep.status} polls={rep.slow_lookbacks / (reps + int(os.environ.get('QO_WARM', '3'))):.0f} ok={ok}", flush=True)
