# Per-decode HBM traffic from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
# of `bench.py --workload W`: bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per decode
# (FETCH_SIZE in KiB; gfx950 counts half the bytes of wide streaming reads, see
# MI355X_MICROARCH.md "HBM"), summed over the kernels of one decode and averaged
# over the traced decodes.
# Usage: python scripts/pmc_traffic.py <out.json> <workload>=<fetch_dir>,<write_dir> ...
# (env PMC_CMD: the profiled command, for the record; default the bench.py line)
import csv, glob, json, os, sys, collections

out_path = sys.argv[1]
try:
    res = json.load(open(out_path))
except (OSError, ValueError):
    res = {}
for arg in sys.argv[2:]:
    wl, dirs = arg.split("=")
    fdir, wdir = dirs.split(",")
    per = {}
    for name, d in (("FETCH_SIZE", fdir), ("WRITE_SIZE", wdir)):
        sums = collections.defaultdict(float)  # kernel name -> sum of the counter
        counts = collections.defaultdict(int)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = row.get("Kernel_Name", "")
                if "gh::" not in k or row["Counter_Name"] != name:
                    continue
                kk = k.split("(")[0].replace("void ", "")
                sums[kk] += float(row["Counter_Value"])
                counts[kk] += 1
        per[name] = {k: sums[k] / counts[k] for k in sums}  # KiB per dispatch of each kernel
    fetch = sum(per["FETCH_SIZE"].values())
    write = sum(per["WRITE_SIZE"].values())
    res[wl] = {
        "bytes_per_launch": (2 * fetch + write) * 1024,
        "fetch_size_kib_per_decode": fetch,
        "write_size_kib_per_decode": write,
        "kernels": sorted(per["FETCH_SIZE"]),
        "round": int(os.environ.get("PMC_ROUND", "0")) or None,
        "source": f"{fdir.rstrip('/')}+{os.path.basename(wdir.rstrip('/'))}: "
                  "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of "
                  + os.environ.get("PMC_CMD", f"`python3 bench.py --workload {wl.split('_')[0]} --cpu-sample 0 --no-copy`")
                  + "; "
                  "bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 "
                  "per decode, summed over its kernels (gfx950 FETCH_SIZE halves wide streaming reads)",
    }
json.dump(res, open(out_path, "w"), indent=1)
print(json.dumps(res, indent=1))
