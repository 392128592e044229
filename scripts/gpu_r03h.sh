#!/bin/bash
# round-3 evidence after the tile-kernel changes: smoke, default bench line (cfg4 + CPU
# baselines + e2e), bench lines cfg2/cfg3/cfg5, dist1 rehearsal, rocprofv3 kernel stats
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03h; mkdir -p $O; export TMPDIR=/tmp
step smoke 300 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench-cfg4 600 $O/bench_cfg4.err python bench.py --out-json $O/bench_cfg4.json || exit 1
cat $O/bench_cfg4.json
for w in cfg2 cfg3 cfg5; do
  step bench-$w 400 $O/bench_$w.err python bench.py --workload $w --cpu-sample 0 --no-e2e --out-json $O/bench_$w.json || exit 1
done
step dist1 400 $O/bench_dist1.err python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --force-dist --steps 10 --warmup 3 --out-json $O/bench_dist1.json || exit 1
for w in cfg4 cfg3 cfg5 cfg2; do
  step prof-$w 400 $O/prof_$w.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py --workload $w --cpu-sample 0 --no-copy --no-e2e || exit 1
done
find $O -name "*kernel_stats.csv" | sort | while read f; do echo "== $f"; cut -d, -f1-6 "$f" | head -5; done
echo done
