# Kernel time against the number of back-to-back decodes (clock behaviour under sustained
# load): one context, decode batches of 3, 20, 100 and 400 launches, average kernel ms each.
# Usage: python scripts/reps.py name:N:r
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'cse375-finalproj-huffman-decoding_amd'))
import numpy as np, gaphuff as gh
name, n, r = sys.argv[1].split(":"); n = int(n); r = float(r)
data = gh.generate(375, r, n); img = gh.encode(data); s = gh.parse(img)
alg = 4 * s.w + 4 * ((s.g + 7) // 8) + s.n
d = gh.Decoder(0); d.load(s)
for _ in range(3): d.decode(timed=False)
d.report()
for reps in (3, 20, 100, 400, 3):
    time.sleep(0.5)  # let the clock recover
    d.reset_timing()
    t0 = time.perf_counter()
    for _ in range(reps): d.decode()
    rep = d.report()
    wall = (time.perf_counter() - t0) * 1e3 / reps
    print(f"{name} reps={reps:4d} kernel_ms={rep.kernel_ms:.4f} wall_ms_per={wall:.4f} frac={alg / rep.kernel_ms / 1e6 / 8000:.4f}", flush=True)
ok = bool(np.array_equal(d.download(s.n), data))
print("bitexact", ok)
