# Per-phase timing of the tile kernel from a GH_TILE_STAMPS build (make variant V=st
# VFLAGS=-DGH_TILE_STAMPS=1): decodes a workload with that library, reads the last
# decode's s_memtime deltas (waves 0 and 4 of every workgroup, first 128 iterations)
# and prints the mean cycles per phase, by workgroup half (dispatch slot) and wave.
# Usage: python scripts/stamps.py [name:N:r] [lib-suffix]
import os, subprocess, sys, tempfile
import numpy as np

here = os.path.dirname(os.path.abspath(__file__))
wl = sys.argv[1] if len(sys.argv) > 1 else "cfg4:1000000000:0.1"
suffix = sys.argv[2] if len(sys.argv) > 2 else "st"
out = os.path.join(tempfile.gettempdir(), f"gh_stamps_{os.getpid()}.bin")
lib = os.path.join(here, "..", "cse375-finalproj-huffman-decoding_amd", "lib", f"libgaphuff_{suffix}.so")
env = dict(os.environ, GAPHUFF_LIB=lib, GH_STAMPS_OUT=out)
r = subprocess.run([sys.executable, os.path.join(here, "quick_one.py"), wl, "3"], env=env, capture_output=True,
                   text=True, timeout=300)
print(r.stdout.strip(), r.stderr.strip()[-500:])
a = np.fromfile(out, dtype=np.uint32)
os.unlink(out)
grid = int(dict(x.split("=", 1) for x in r.stdout.split() if "=" in x)["grid"])
a = a[:grid * 2 * 128 * 8].reshape(grid, 2, 128, 8).astype(np.float64)  # (then the chain times)
names = ["load wait", "decode", "scans+arrive", "prefix", "copy-out", "stage", "-", "-"]
valid = a.sum(axis=3) > 0
valid[0] = False  # workgroup 0 leads the rounds
print(f"grid {grid}, stamped iterations {int(valid.sum())}")
for label, sel in [("all", np.ones(grid, bool)), ("WG < grid/2", np.arange(grid) < grid // 2),
                   ("WG >= grid/2", np.arange(grid) >= grid // 2)]:
    for wv in (0, 1):
        m = valid[:, wv, :] & sel[:, None]
        d = a[:, wv, :, :][m]
        if d.size == 0:
            continue
        tot = d.sum(axis=1).mean()
        parts = "  ".join(f"{n} {d[:, i].mean():7.0f}" for i, n in enumerate(names))
        print(f"{label:13s} wave {4 * wv}: total {tot:7.0f} | {parts}")
# per-workgroup sums over its iterations (wave 0): a grid whose rounds wait for the
# slowest workgroup shows it as the workgroups that never wait for a prefix
w0 = a[:, 0, :, :] * valid[:, 0, :, None]
busy = w0.sum(axis=(1, 2)) - w0[:, :, 3].sum(axis=1)
pref = w0[:, :, 3].sum(axis=1)
iters = valid[:, 0, :].sum(axis=1)
sel = iters > 0
q = [0, 1, 10, 50, 90, 99, 100]
print("per-WG iterations   ", np.percentile(iters[sel], q).round(0))
print("per-WG busy cycles  ", np.percentile(busy[sel], q).round(-3))
print("per-WG prefix cycles", np.percentile(pref[sel], q).round(-3))
slow = np.argsort(busy[sel])[-8:]
print("slowest WGs (busy)  ", np.nonzero(sel)[0][slow], busy[sel][slow].round(-3))

# by XCD (blocks are dealt round-robin over the 8 XCDs: block b on XCD b mod 8, as
# observed; which physical XCD is not fixed) and, for the slowest / fastest workgroups,
# the phases that differ
blk = np.arange(grid)
for x in range(8):
    m = sel & (blk % 8 == x)
    if m.any():
        ph = (w0[m].sum(axis=1) / iters[m][:, None]).mean(axis=0)
        print(f"XCD {x}: busy/iter {(busy[m] / iters[m]).mean():7.0f}  " +
              "  ".join(f"{n} {ph[i]:6.0f}" for i, n in enumerate(names[:6])))
for label, idx in [("slowest 8", np.nonzero(sel)[0][np.argsort(busy[sel])[-8:]]),
                   ("fastest 8", np.nonzero(sel)[0][np.argsort(busy[sel])[:8]])]:
    ph = (w0[idx].sum(axis=1) / iters[idx][:, None]).mean(axis=0)
    print(f"{label}: " + "  ".join(f"{n} {ph[i]:6.0f}" for i, n in enumerate(names[:6])))
