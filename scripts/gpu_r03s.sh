#!/bin/bash
# tile-kernel knobs after the scan move: prefix load after decode group 1 / 3 (default 2),
# copy-out NS = 3 (default 2); cfg4, four passes
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03s; mkdir -p $O; export TMPDIR=/tmp
step cmp4 600 $O/cmp4.log python -u scripts/cmp_libs.py "cfg4:1000000000:0.1" base midg1 midg3 ns3 base midg1 midg3 ns3 base midg1 midg3 ns3 base midg1 midg3 ns3 || exit 1
cat $O/cmp4.log
