#!/bin/bash
# long codes (16-bit geometric streams) through the wave split's fallback kernels, with
# the fixed-store count kernel
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03t; mkdir -p $O; export TMPDIR=/tmp
step longcodes 500 $O/longcodes.txt python -u scripts/time_longcodes.py || exit 1
cat $O/longcodes.txt
