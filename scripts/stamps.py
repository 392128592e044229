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
raw = np.fromfile(out, dtype=np.uint8)
os.unlink(out)
if os.environ.get("STAMPS_KEEP"):  # the raw dump, for offline analysis
    raw.tofile(os.environ["STAMPS_KEEP"])
a = raw.view(np.uint32)
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

# ---- hand-off chain (100 MHz s_memrealtime): aggregate left -> round published (leader
# latency) -> prefix obtained by the copying wave 0 (consumer latency); per-workgroup clock
ntiles = int(dict(x.split("=", 1) for x in r.stdout.split() if "=" in x).get("tiles", 0) or 0)
t = raw[32 * grid * 2 * 128:].view(np.uint64)
if ntiles == 0:  # (quick_one does not print the tile count: from the table sizes)
    ntiles = (t.size - 64 - 4 * 1024 - 4 * grid) // 3
agg = t[:ntiles].astype(np.float64)
got = (t[ntiles:2 * ntiles] & ((1 << 63) - 1)).astype(np.float64)
D = grid - 1
nr = (ntiles + D - 1) // D
pub = t[2 * ntiles:2 * ntiles + nr].astype(np.float64)
lat_lead, lat_cons, spread = [], [], []
for rr in range(nr):
    lo, hi = rr * D, min(ntiles, (rr + 1) * D)
    ag = agg[lo:hi]
    if pub[rr] == 0 or (ag == 0).any():
        continue
    lat_lead.append((pub[rr] - ag.max()) * 0.01)
    spread.append((ag.max() - np.median(ag)) * 0.01)
    g2 = got[lo:hi]
    g2 = g2[g2 > 0]
    lat_cons.extend(((g2 - pub[rr]) * 0.01).tolist())
q = [10, 50, 90, 99]
if lat_lead:
    print("round: last aggregate - median aggregate us", np.percentile(spread, q).round(2))
    print("round: published - last aggregate us (leader)", np.percentile(lat_lead, q).round(2))
    lc = np.array(lat_cons)
    print("prefix obtained - published us (consumers; < 0: seen by its own early load)",
          np.percentile(lc, q).round(2))
wr = t[3 * ntiles + 64 + 4 * 1024:3 * ntiles + 64 + 4 * 1024 + 4 * grid].reshape(grid, 4).astype(np.float64)
okw = (wr[:, 3] > wr[:, 1]) & (np.arange(grid) > 0)
clk = (wr[okw, 2] - wr[okw, 0]) / (wr[okw, 3] - wr[okw, 1]) / 10.0
print("per-WG clock GHz pct", np.percentile(clk, [0, 10, 50, 90, 100]).round(3))
blk2 = np.arange(grid)[okw]
for x in range(8):
    m = blk2 % 8 == x
    print(f"  XCD {x}: clock {clk[m].mean():.3f} GHz, span us {((wr[okw][m, 3] - wr[okw][m, 1]) * 0.01).mean():.1f}")
busy_ok = busy[okw] if busy.size == grid else None
if busy_ok is not None:
    print("corr(busy, clock)", np.corrcoef(busy_ok, clk)[0, 1].round(3))
