#!/bin/bash
# Round-2 first GPU pass: GPU tests (not slow), smoke, the default bench line (cfg4 with
# the CPU baselines), cfg3, and a rocprofv3 kernel-trace summary of the cfg4 bench.
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${R:-r02a}
mkdir -p $O
export TMPDIR=/tmp
step pytest 900 $O/pytest_gpu.log python -u -m pytest tests -m "gpu and not slow" -q -rf --timeout 180 --timeout-method thread
tail -15 $O/pytest_gpu.log
step smoke 300 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()"; cat $O/smoke.log
step bench-cfg4 600 $O/bench_cfg4.err python bench.py --out-json $O/bench_cfg4.json
cat $O/bench_cfg4.json; tail -3 $O/bench_cfg4.err
step bench-cfg3 400 $O/bench_cfg3.err python bench.py --workload cfg3 --cpu-sample 0 --out-json $O/bench_cfg3.json
cat $O/bench_cfg3.json
step prof-cfg4 400 $O/prof_cfg4.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg4 -o run -- python3 bench.py --cpu-sample 0 --no-copy
find $O/prof_cfg4 -name "*kernel_stats.csv" -exec head -5 {} \;
echo done
