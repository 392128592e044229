#!/bin/bash
# GPU tests (not slow) + cfg4/cfg3/cfg5 timings
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03f; mkdir -p $O
export TMPDIR=/tmp
step pytest 900 $O/pytest_gpu.log python -u -m pytest tests -m "gpu and not slow" -q -rf --timeout 180 --timeout-method thread
tail -5 $O/pytest_gpu.log
for w in cfg4:1000000000:0.1 cfg4:1000000000:0.1 cfg3:1000000000:0.9 cfg5:1000000000:0.5; do
  step q 120 $O/q.log python -u scripts/quick_one.py $w 20 || exit 1; cat $O/q.log
done
