# Prefix-chain timing of the tile kernel from a GH_TILE_STAMPS build: per round, when its
# tiles' aggregates left (100 MHz clock), when the leader published the round, when wave
# 0 of each decoding workgroup obtained each tile's prefix (and whether it polled).
# Usage: python scripts/chain.py [name:N:r] [lib-suffix]
import os, subprocess, sys, tempfile
import numpy as np

here = os.path.dirname(os.path.abspath(__file__))
wl = sys.argv[1] if len(sys.argv) > 1 else "cfg4:1000000000:0.1"
suffix = sys.argv[2] if len(sys.argv) > 2 else "st"
out = os.path.join(tempfile.gettempdir(), f"gh_chain_{os.getpid()}.bin")
lib = os.path.join(here, "..", "cse375-finalproj-huffman-decoding_amd", "lib", f"libgaphuff_{suffix}.so")
env = dict(os.environ, GAPHUFF_LIB=lib, GH_STAMPS_OUT=out)
r = subprocess.run([sys.executable, os.path.join(here, "quick_one.py"), wl, "3"], env=env, capture_output=True,
                   text=True, timeout=300)
print(r.stdout.strip(), r.stderr.strip()[-500:])
kv = dict(x.split("=", 1) for x in r.stdout.split() if "=" in x)
grid = int(kv["grid"])
raw = np.fromfile(out, dtype=np.uint8)
os.unlink(out)
t = raw[32 * grid * 2 * 128:].view(np.uint64)
ntiles = (t.size - 64) // 3
D = grid - 1
nr = (ntiles + D - 1) // D
agg = t[:ntiles].astype(np.float64)
got_raw = t[ntiles:2 * ntiles]
polled = (got_raw >> np.uint64(63)).astype(bool)
got = (got_raw & np.uint64((1 << 63) - 1)).astype(np.float64)
rnd = t[2 * ntiles:2 * ntiles + nr].astype(np.float64)
t0 = agg[agg > 0].min()
us = 0.01  # 100 MHz ticks -> us
rows = []
for q in range(nr):
    a = agg[q * D:min(ntiles, (q + 1) * D)]
    g = got[q * D:min(ntiles, (q + 1) * D)]
    rows.append((q, (a.min() - t0) * us, (np.median(a) - t0) * us, (a.max() - t0) * us, (rnd[q] - t0) * us,
                 (np.median(g[g > 0]) - t0) * us if (g > 0).any() else np.nan))
rows = np.array(rows)
print(f"tiles {ntiles}, grid {grid}, rounds {nr}; times in us from the first aggregate")
print(" round  agg_min  agg_med  agg_max  published  got_med | spread  lead_lat  period")
for q in list(range(0, min(nr, 6))) + list(range(nr // 2, nr // 2 + 4)) + list(range(max(0, nr - 4), nr)):
    _, amin, amed, amax, pub, gmed = rows[q]
    per = rows[q, 4] - rows[q - 1, 4] if q else np.nan
    print(f"{q:6d} {amin:8.2f} {amed:8.2f} {amax:8.2f} {pub:10.2f} {gmed:8.2f} | {amax - amin:6.2f} {pub - amax:9.2f} {per:7.2f}")
mid = rows[2:-2]
print(f"median over rounds: spread (agg max - min) {np.median(mid[:, 3] - mid[:, 1]):.2f} us, "
      f"(agg max - median) {np.median(mid[:, 3] - mid[:, 2]):.2f} us, leader (published - agg max) "
      f"{np.median(mid[:, 4] - mid[:, 3]):.2f} us, period {np.median(np.diff(rows[:, 4])):.2f} us, "
      f"got - published {np.median(mid[:, 5] - mid[:, 4]):.2f} us")
print(f"wave-0 prefix checks that polled: {polled.mean() * 100:.1f} %")
# per decoding workgroup: how late its aggregates are against each round's median
late = np.full((nr, D), np.nan)
for q in range(2, nr - 2):
    a = agg[q * D:min(ntiles, (q + 1) * D)]
    late[q, :a.size] = (a - np.median(a)) * us
pw = np.nanmedian(late, axis=0)
order = np.argsort(pw)
print("per-WG median lateness (us): min %.2f  p10 %.2f  p50 %.2f  p90 %.2f  max %.2f" % tuple(
    np.percentile(pw, [0, 10, 50, 90, 100])))
print("latest WGs (block = index + 1):", [(int(b) + 1, round(float(pw[b]), 2)) for b in order[-10:]])
print("earliest WGs:", [(int(b) + 1, round(float(pw[b]), 2)) for b in order[:5]])
# per round, which WG was last; how often the same
lastw = [int(np.nanargmax(late[q])) for q in range(2, nr - 2)]
vals, cnts = np.unique(lastw, return_counts=True)
print("last-arriving WG per round (block, rounds):", sorted(zip((vals + 1).tolist(), cnts.tolist()), key=lambda x: -x[1])[:8])
