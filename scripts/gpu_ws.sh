#!/bin/bash
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${R:-ws}
mkdir -p $O
step wstest 400 $O/wstest.log python -u -m pytest tests/test_gpu_decode.py -q -x -k "lean or wave or shard or generated" --timeout 120 --timeout-method thread; tail -5 $O/wstest.log
step env 600 $O/env.log python scripts/cmp_env.py "${WL:-cfg3:1000000000:0.9,cfg2:100000000:0.5,cfg5:1000000000:0.5}" "GH_MODE=msplit" "GH_MODE=wsplit" "$@"; cat $O/env.log
