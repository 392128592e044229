# Time decode variants on one config: python scripts/variants.py cfg4:1000000000:0.1 "GH_MODE=fused" "GH_MODE=tile GH_LGR=3" ...
# Each variant = space-separated env assignments applied before load.  Prints kernel ms,
# algorithmic GB/s, roofline fraction, slow look-backs and bit-exactness.
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'cse375-finalproj-huffman-decoding_amd'))
import numpy as np, gaphuff as gh
name, n, r = sys.argv[1].split(":"); n = int(n); r = float(r)
data = gh.generate(375, r, n); img = gh.encode(data); s = gh.parse(img)
alg = 4 * s.w + 4 * ((s.g + 7) // 8) + s.n
for v in sys.argv[2:] or [""]:
    # the environment of this process carries the variant (set by scripts/gpu_v.sh)
    d = gh.Decoder(0); d.load(s)
    for _ in range(3): d.decode(timed=False)
    d.report(); d.reset_timing()
    for _ in range(10): d.decode()
    rep = d.report()
    ok = np.array_equal(d.download(s.n), data) and rep.status == 0
    ms = rep.kernel_ms
    tag = v.replace(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cse375-finalproj-huffman-decoding_amd", "lib") + "/", "")
    print(f"{name} [{tag[-40:]:40s}] mode={gh.MODE_NAMES.get(rep.mode)} K={rep.lut_bits} grid={rep.grid} ms={ms:.3f} "
          f"dec={n/ms/1e6:.0f} GB/s frac={alg/ms/1e6/8000:.3f} slow_lb={rep.slow_lookbacks} st={rep.status} ok={ok}", flush=True)
    d.close()
