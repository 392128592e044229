# Diagnostic: per-phase cycle shares of the decode kernel (GH_STAMPS build).
import ctypes, os, sys
here = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("GAPHUFF_LIB", os.path.join(here, "..", "cse375-finalproj-huffman-decoding_amd", "lib", "libgaphuff_stamps.so"))
sys.path.insert(0, os.path.join(here, "..", "cse375-finalproj-huffman-decoding_amd"))
import numpy as np, gaphuff as gh
L = gh.lib(); L.gh_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]; L.gh_debug_stamps.restype = ctypes.c_int
names = ["decode", "bar0", "clr+bar1", "resolve", "bar2", "copyout", "stage", "memwait", "-", "top"]
cfgs = [a.split(":") for a in sys.argv[1:]] or [["cfg4", "1000000000", "0.1"], ["cfg3", "1000000000", "0.9"]]
for name, n, r in cfgs:
    n = int(n); r = float(r)
    data = gh.generate(375, r, n); img = gh.encode(data); s = gh.parse(img)
    d = gh.Decoder(0); d.load(s)
    for _ in range(3): d.decode()
    rep = d.report()
    buf = np.zeros((rep.grid, 16), dtype=np.uint64)
    nb = L.gh_debug_stamps(d._h, ctypes.c_void_p(buf.ctypes.data), rep.grid)
    tot = buf[:, :10].astype(np.float64)
    per_block = tot.sum(1)
    ok = np.array_equal(d.download(s.n), data)
    print(f"{name} K={rep.lut_bits} grid={rep.grid} tiles={rep.tiles} kernel_ms={rep.kernel_ms:.3f} ok={ok}")
    print(f"  per-block total ticks: mean {per_block.mean():.0f} -> ticks/ms {per_block.mean()/rep.kernel_ms:.0f}")
    tiles_per_block = rep.tiles / rep.grid
    for i, nm in enumerate(names):
        print(f"  {nm:9s} {100*tot[:, i].sum()/tot.sum():6.2f}%  per tile {tot[:, i].mean()/tiles_per_block:9.0f} ticks")
    d.close()
