#!/bin/bash
# round-3 evidence after the count-kernel change: full GPU suite, smoke, wave-split bench
# lines cfg3/5/2 and their kernel stats
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03l; mkdir -p $O; export TMPDIR=/tmp
step pytest 900 $O/pytest.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step smoke 300 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for w in cfg3 cfg5 cfg2; do
  step bench-$w 400 $O/bench_$w.err python bench.py --workload $w --cpu-sample 0 --no-e2e --out-json $O/bench_$w.json || exit 1
  step prof-$w 400 $O/prof_$w.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py --workload $w --cpu-sample 0 --no-copy --no-e2e || exit 1
done
for w in cfg3 cfg5 cfg2; do python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', d['roofline']['kernel_ms'], d['value'], d['roofline']['frac'], d['roofline']['copy_frac'], d['bitexact'])"; done
