# Summarise rocprofv3 PMC passes (per kernel dispatch averages) for the decode kernel.
import csv, glob, os, sys, collections
root = sys.argv[1]
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if "gh_decode" not in row.get("Kernel_Name", ""):
            continue
        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
dur = []
for f in glob.glob(os.path.join(root, "*", "**", "*kernel_trace.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if "gh_decode" in row.get("Kernel_Name", ""):
            dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
out = {k: sum(v) / len(v) for k, v in vals.items()}
for k in sorted(out):
    print(f"{k:28s} {out[k]:16.0f}")
if dur:
    print("kernel_us(avg over traced dispatches)", sum(dur) / len(dur), "n", len(dur))
