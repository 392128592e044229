#!/bin/bash
set -o pipefail
O=gpurun_out/t1k; mkdir -p $O
GH_MODE=tile timeout -k 10 300 python -u scripts/cmp_libs.py cfg4:1000000000:0.1 base tp t1k t1kp > $O/cmp.log 2>&1; rc=$?
cat $O/cmp.log; exit $rc
