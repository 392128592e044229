#!/bin/bash
set -o pipefail
O=gpurun_out/wsprio; mkdir -p $O
timeout -k 10 500 python -u scripts/cmp_libs.py cfg3:1000000000:0.9,cfg5:1000000000:0.5,cfg2:100000000:0.5 base wp2 wp4 bf0 > $O/cmp.log 2>&1; rc=$?
cat $O/cmp.log; exit $rc
