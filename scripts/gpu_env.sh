#!/bin/bash
# WL="cfg3:1000000000:0.9" bash scripts/gpu_env.sh "" "GH_MODE=msplit" ...
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${R:-env}
mkdir -p $O
step env 900 $O/env.log python scripts/cmp_env.py "${WL:-cfg3:1000000000:0.9}" "$@"; cat $O/env.log
