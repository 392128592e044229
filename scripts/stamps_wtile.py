# Diagnostic: per-phase cycles per iteration of the wave-tile kernel (GH_STAMPS build),
# averaged over all waves.  Usage: python scripts/stamps_wtile.py cfg:n:r
import ctypes, os, sys
here = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("GAPHUFF_LIB", os.path.join(here, "..", "cse375-finalproj-huffman-decoding_amd", "lib", "libgaphuff_stamps.so"))
os.environ.setdefault("GH_MODE", "wtile")
sys.path.insert(0, os.path.join(here, "..", "cse375-finalproj-huffman-decoding_amd"))
import numpy as np, gaphuff as gh
L = gh.lib(); L.gh_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]; L.gh_debug_stamps.restype = ctypes.c_int
names = ["decode", "scan+arrive", "lead", "prefix-wait", "copyout", "stage", "load+top"]
name, n, r = sys.argv[1].split(":"); n = int(n); r = float(r)
data = gh.generate(375, r, n); img = gh.encode(data); s = gh.parse(img)
d = gh.Decoder(0); d.load(s)
for _ in range(3): d.decode()
d.report(); d.reset_timing()
for _ in range(5): d.decode()
rep = d.report()
rows = rep.grid * 8
buf = np.zeros((rows, 16), dtype=np.uint64)
nr = L.gh_debug_stamps(d._h, ctypes.c_void_p(buf.ctypes.data), rows)
tot = buf[:nr, :7].astype(np.float64)
iters = rep.tiles / rep.grid + 2
ok = np.array_equal(d.download(s.n), data)
print(f"{name} grid={rep.grid} tiles={rep.tiles} kernel_ms={rep.kernel_ms:.3f} ok={ok} rows={nr}")
print("   " + "  ".join(f"{names[i]}={tot[:, i].mean() / iters:.0f}" for i in range(7)) +
      f"  (cycles/iter, mean over waves; total/iter {tot.sum(1).mean() / iters:.0f}; max wave total {tot.sum(1).max() / iters:.0f})", flush=True)
for w in range(8):
    sel = tot[w::8]
    print(f"   wave {w}: " + " ".join(f"{sel[:, i].mean() / iters:6.0f}" for i in range(7)))
d.close()
