import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'cse375-finalproj-huffman-decoding_amd'))
import numpy as np, gaphuff as gh
for name, n, r in [('cfg2', 10**8, 0.5), ('cfg3', 10**9, 0.9), ('cfg4', 10**9, 0.1)]:
    t = time.time(); data = gh.generate(375, r, n); tg = time.time() - t
    t = time.time(); img = gh.encode(data); te = time.time() - t
    s = gh.parse(img)
    d = gh.Decoder(0); d.load(s)
    for _ in range(3): d.decode(timed=False)
    d.report(); d.reset_timing()
    for _ in range(10): d.decode()
    rep = d.report()
    out = d.download(s.n)
    ok = np.array_equal(out, data)
    ms = rep.kernel_ms
    alg = 4*s.w + 4*((s.g+7)//8) + s.n
    print(f"{name}: N={n} W={s.w} G={s.g} K={rep.lut_bits} grid={rep.grid} ms={ms:.3f} dec={n/ms/1e6:.1f} GB/s alg={alg/ms/1e6:.1f} GB/s frac={alg/ms/1e6/8000:.3f} ok={ok} gen={tg:.1f}s enc={te:.1f}s", flush=True)
    d.close(); del data, img, out
