#!/bin/bash
# round-3 evidence refresh after the DPP wave-sum change: default bench line (cfg4 + CPU
# baselines + e2e) and rocprofv3 kernel stats for cfg4
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03i; mkdir -p $O; export TMPDIR=/tmp
step bench-cfg4 600 $O/bench_cfg4.err python bench.py --out-json $O/bench_cfg4.json || exit 1
cat $O/bench_cfg4.json
step prof-cfg4 400 $O/prof_cfg4.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg4 -o run -- python3 bench.py --workload cfg4 --cpu-sample 0 --no-copy --no-e2e || exit 1
find $O -name "*kernel_stats.csv" | sort | while read f; do echo "== $f"; cut -d, -f1-6 "$f" | head -5; done
echo done
