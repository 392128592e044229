#!/bin/bash
# Refresh the r=0.5 evidence after the write-LUT width change: cfg2 / cfg5 bench lines,
# cfg2 kernel stats and FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r02e; mkdir -p $O; export TMPDIR=/tmp
for w in cfg2 cfg5; do
  step bench-$w 400 $O/bench_$w.err python bench.py --workload $w --cpu-sample 0 --out-json $O/bench_$w.json || exit 1
done
step rocprof-cfg2 300 $O/prof_cfg2.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg2 -o run -- python3 bench.py --workload cfg2 --cpu-sample 0 --no-copy || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc-$c 300 $O/pmc_${c}_cfg2.log rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${c}_cfg2 -o run -- python3 bench.py --workload cfg2 --cpu-sample 0 --no-copy || exit 1
done
python3 scripts/pmc_traffic.py $O/pmc_traffic.json cfg2_100000000_n1=$O/pmc_FETCH_SIZE_cfg2,$O/pmc_WRITE_SIZE_cfg2 > /dev/null
echo done
