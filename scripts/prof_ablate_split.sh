#!/bin/bash
# split-mode per-kernel times with the decode ablated (stamps build)
set -o pipefail
export TMPDIR=/tmp
export GAPHUFF_LIB=$PWD/cse375-finalproj-huffman-decoding_amd/lib/libgaphuff_stamps.so
O=gpurun_out/pabl${TAG}
mkdir -p $O
for a in 0 8; do
for c in cfg4:1000000000:0.1 cfg3:1000000000:0.9; do
  n=$(echo $c | cut -d: -f1)
  GH_ABLATE=$a timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${n}_$a -o run -- python3 scripts/quick_one.py $c 5 > $O/${n}_$a.log 2>&1 || exit 1
  echo "== $n ablate=$a"; python3 -c "
import csv
for r in csv.DictReader(open('$O/${n}_$a/run_kernel_stats.csv')):
    if 'gh_' in r['Name']: print(r['Name'][:40], round(float(r['AverageNs'])/1e3,1))
"
done; done
