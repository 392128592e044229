#!/bin/bash
# after removing the retired decode structures: GPU tests (not slow) + quick timings
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03d; mkdir -p $O
export TMPDIR=/tmp
step pytest 900 $O/pytest_gpu.log python -u -m pytest tests -m "gpu and not slow" -x -q -rf --timeout 180 --timeout-method thread
tail -8 $O/pytest_gpu.log
step q4 200 $O/q.log python -u scripts/quick_one.py cfg4:1000000000:0.1 20 || exit 1
step q3 200 $O/q3.log python -u scripts/quick_one.py cfg3:1000000000:0.9 20 || exit 1
step q5 200 $O/q5.log python -u scripts/quick_one.py cfg5:1000000000:0.5 20 || exit 1
cat $O/q.log $O/q3.log $O/q5.log
