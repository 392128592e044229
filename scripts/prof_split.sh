#!/bin/bash
# Per-kernel times (split mode) for cfg4 / cfg3 / cfg2.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/psplit${TAG}
mkdir -p $O
for c in cfg4:1000000000:0.1 cfg3:1000000000:0.9 cfg2:100000000:0.5; do
  n=$(echo $c | cut -d: -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 scripts/quick_one.py $c 5 > $O/$n.log 2>&1 || exit 1
  echo "== $n"; grep -h "gh_\|Name" $O/$n/run_kernel_stats.csv | cut -d, -f1-4
done
