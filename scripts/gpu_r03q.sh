#!/bin/bash
# tile kernel: the three wave scans issued together (scan3) vs one after another (base), cfg4
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03q; mkdir -p $O; export TMPDIR=/tmp
step cmp4 600 $O/cmp4.log python -u scripts/cmp_libs.py "cfg4:1000000000:0.1" scan3 base scan3 base scan3 base scan3 base || exit 1
cat $O/cmp4.log
