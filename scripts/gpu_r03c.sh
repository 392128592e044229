#!/bin/bash
# wave split for every non-grouped code (canonical fallback for long / incomplete codes)
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03c; mkdir -p $O
export TMPDIR=/tmp
step pytest 900 $O/pytest_gpu.log python -u -m pytest tests -m "gpu and not slow" -q -rf --timeout 180 --timeout-method thread
tail -8 $O/pytest_gpu.log
step longcodes 300 $O/longcodes.txt python -u scripts/time_longcodes.py
cat $O/longcodes.txt
