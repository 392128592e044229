#!/bin/bash
# round-3 evidence for the wave split after the e-window change: bench lines cfg2/3/5 and
# rocprofv3 kernel stats
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03k; mkdir -p $O; export TMPDIR=/tmp
for w in cfg3 cfg5 cfg2; do
  step bench-$w 400 $O/bench_$w.err python bench.py --workload $w --cpu-sample 0 --no-e2e --out-json $O/bench_$w.json || exit 1
  step prof-$w 400 $O/prof_$w.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py --workload $w --cpu-sample 0 --no-copy --no-e2e || exit 1
done
for w in cfg3 cfg5 cfg2; do python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', d['roofline']['kernel_ms'], d['value'], d['roofline']['frac'], d['roofline']['copy_frac'], d['bitexact'])"; done
find $O -name "*kernel_stats.csv" | sort | while read f; do echo "== $f"; cut -d, -f1-4 "$f" | head -6; done
