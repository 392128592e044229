#!/bin/bash
# GPU tests (not slow)
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03e; mkdir -p $O
export TMPDIR=/tmp
step pytest 900 $O/pytest_gpu.log python -u -m pytest tests -m "gpu and not slow" -q -rf --timeout 180 --timeout-method thread
tail -8 $O/pytest_gpu.log
