#!/bin/bash
# final round-3 check of the committed library: full GPU suite, smoke, default bench line
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03r; mkdir -p $O; export TMPDIR=/tmp
step pytest 900 $O/pytest.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step smoke 300 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
cat $O/smoke.log | tail -2
step bench 600 $O/bench.err python bench.py --out-json $O/bench_cfg4.json || exit 1
python3 -c "import json; d=json.load(open('$O/bench_cfg4.json')); r=d['roofline']; print('cfg4', d['ms_per_step'], r['kernel_ms'], r['frac'], d['bitexact'])"
