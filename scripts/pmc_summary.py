# Summarise rocprofv3 PMC passes: per-kernel dispatch averages of every counter, plus
# the kernel-trace duration.  Usage: python scripts/pmc_summary.py <dir> [name-filter]
import csv, glob, os, sys, collections
root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else "gh_"


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "")[:60]


vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if filt not in k:
            continue
        vals[short(k)][row["Counter_Name"]].append(float(row["Counter_Value"]))
dur = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if filt in k:
            dur[short(k)].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
for kern in sorted(set(vals) | set(dur)):
    print(f"== {kern}")
    for c in sorted(vals[kern]):
        v = vals[kern][c]
        print(f"  {c:28s} {sum(v) / len(v):16.0f}")
    d = dur[kern]
    if d:
        print(f"  kernel_us(avg) {sum(d) / len(d):.1f} n {len(d)}")
