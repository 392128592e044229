# Per-dispatch durations of gh_tile_kernel from a rocprofv3 kernel trace, in launch order,
# summarised in windows (clock behaviour over a burst).  Usage: python scripts/trace_series.py DIR
import csv, glob, os, sys
import numpy as np
rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if (sys.argv[2] if len(sys.argv) > 2 else "gh_tile_kernel") in r.get("Kernel_Name", ""):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
rows.sort()
d = np.array([(e - s) / 1e3 for s, e in rows])
t = np.array([(s - rows[0][0]) / 1e6 for s, e in rows])
print(f"{d.size} dispatches")
i = 0
while i < d.size:
    j = i + 1
    while j < d.size and t[j] - t[j - 1] < 50:  # a burst: gaps under 50 ms
        j += 1
    b = d[i:j]
    w = max(1, b.size // 8)
    parts = " ".join(f"{b[k:k + w].mean():.0f}" for k in range(0, b.size, w))
    print(f"burst at {t[i]:8.1f} ms: {b.size:4d} launches, mean {b.mean():.1f} us; by window of {w}: {parts}")
    i = j
