#!/bin/bash
set -o pipefail
O=gpurun_out/tq; mkdir -p $O
GH_MODE=tile timeout -k 10 300 python -u scripts/cmp_libs.py cfg4:1000000000:0.1 base np t256 u4t256 > $O/cmp.log 2>&1; rc=$?
cat $O/cmp.log; exit $rc
