#!/bin/bash
# Compare lib variants: WL="cfg4:1000000000:0.1" LIBS="base lag3 top" bash scripts/gpu_cmp.sh
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${R:-cmp}
mkdir -p $O
step cmp 600 $O/cmp.log python scripts/cmp_libs.py "${WL:-cfg4:1000000000:0.1}" ${LIBS:-base}; cat $O/cmp.log
