# Diagnostic: per-phase cycles per iteration of the wave-tile kernel (GH_STAMPS build),
# averaged over all waves.  Usage: python scripts/stamps_wtile.py cfg:n:r
import ctypes, os, sys
here = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("GAPHUFF_LIB", os.path.join(here, "..", "cse375-finalproj-huffman-decoding_amd", "lib", "libgaphuff_stamps.so"))
os.environ.setdefault("GH_MODE", "wtile")
sys.path.insert(0, os.path.join(here, "..", "cse375-finalproj-huffman-decoding_amd"))
import numpy as np, gaphuff as gh
L = gh.lib(); L.gh_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]; L.gh_debug_stamps.restype = ctypes.c_int
names = ["count", "window", "decode", "scan+P", "stage", "copyout", "-"]
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
tot = buf[:nr, :6].astype(np.float64)
iters = rep.tiles / rep.grid
ok = np.array_equal(d.download(s.n), data)
print(f"{name} grid={rep.grid} tiles={rep.tiles} kernel_ms={rep.kernel_ms:.3f} ok={ok} rows={nr}")
print("   " + "  ".join(f"{names[i]}={tot[:, i].mean() / iters:.0f}" for i in range(6)) +
      f"  (cycles/iter, mean over waves; total/iter {tot.sum(1).mean() / iters:.0f}; max wave total {tot.sum(1).max() / iters:.0f})", flush=True)
cnt = buf[:nr, 6:8].astype(np.float64)
print(f"   window polls per wave-iteration {cnt[:, 0].mean() / iters:.3f}, poll rounds per poll {cnt[:, 1].sum() / max(cnt[:, 0].sum(), 1):.2f}")
# per-workgroup busy cycles (count + decode + stage + copy-out, no waits): spread across WGs and by XCD (b mod 8)
busy = (tot[:, 0] + tot[:, 2] + tot[:, 4] + tot[:, 5]).reshape(-1, 8).mean(1) / iters
q = np.percentile(busy, [0, 1, 10, 50, 90, 99, 100])
print("   busy cycles/iter per WG: min/p1/p10/p50/p90/p99/max " + " ".join(f"{x:.0f}" for x in q))
print("   by XCD (b mod 8): " + " ".join(f"{busy[i::8].mean():.0f}" for i in range(8)))
print("   by CU slot (b // 256): " + " ".join(f"{busy[i*256:(i+1)*256].mean():.0f}" for i in range(len(busy) // 256)))
for w in range(8):
    sel = tot[w::8]
    print(f"   wave {w}: " + " ".join(f"{sel[:, i].mean() / iters:6.0f}" for i in range(6)))
d.close()
