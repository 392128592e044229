# Diagnostic: per-phase cycle shares of the tile kernel (GH_STAMPS build), plus
# kernel time under GH_ABLATE settings.  Usage: python scripts/stamps_tile.py cfg:n:r [ablate...]
import ctypes, os, sys
here = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("GAPHUFF_LIB", os.path.join(here, "..", "cse375-finalproj-huffman-decoding_amd", "lib", "libgaphuff_stamps.so"))
os.environ.setdefault("GH_MODE", "tile")
sys.path.insert(0, os.path.join(here, "..", "cse375-finalproj-huffman-decoding_amd"))
import numpy as np, gaphuff as gh
L = gh.lib(); L.gh_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]; L.gh_debug_stamps.restype = ctypes.c_int
names = {9: "top", 0: "decode", 6: "poll", 1: "copyout", 2: "scan+lead", 3: "barrier", 4: "publish", 5: "stage"}
name, n, r = sys.argv[1].split(":"); n = int(n); r = float(r)
data = gh.generate(375, r, n); img = gh.encode(data); s = gh.parse(img)
for ab in (sys.argv[2:] or ["0"]):
    os.environ["GH_ABLATE"] = ab
    d = gh.Decoder(0); d.load(s)
    for _ in range(3): d.decode()
    d.report(); d.reset_timing()
    for _ in range(5): d.decode()
    rep = d.report()
    buf = np.zeros((rep.grid, 16), dtype=np.uint64)
    L.gh_debug_stamps(d._h, ctypes.c_void_p(buf.ctypes.data), rep.grid)
    tot = buf[:, :10].astype(np.float64)
    ok = np.array_equal(d.download(s.n), data)
    st3 = np.zeros(4, dtype=np.uint64)
    L.gh_debug_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.gh_debug_stats(d._h, ctypes.c_void_p(st3.ctypes.data))
    iters = rep.tiles / rep.grid
    print(f"{name} ablate={ab} K={rep.lut_bits} grid={rep.grid} tiles={rep.tiles} kernel_ms={rep.kernel_ms:.3f} "
          f"slow_lb={rep.slow_lookbacks} ok={ok} stats={list(st3)} per launch {[int(x) // 8 for x in st3]}")
    print("   " + "  ".join(f"{names[i]}={tot[:, i].mean() / iters:.0f}" for i in (9, 0, 6, 1, 2, 3, 4, 5)) +
          f"  (cycles/iter, wave 0; total/iter {tot.sum(1).mean() / iters:.0f})", flush=True)
    d.close()
