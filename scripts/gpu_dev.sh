#!/bin/bash
# Development pass: GPU tests (not slow) then env-variant timings.
# WL=... bash scripts/gpu_dev.sh "" "GH_MODE=msplit" ...
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${R:-dev}
mkdir -p $O
step pytest 600 $O/pytest.log python -u -m pytest tests -m "gpu and not slow" -x -q -rf --timeout 120 --timeout-method thread
tail -15 $O/pytest.log
step env 900 $O/env.log python scripts/cmp_env.py "${WL:-cfg3:1000000000:0.9}" "$@"; cat $O/env.log
