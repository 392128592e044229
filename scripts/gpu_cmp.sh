#!/bin/bash
# compare library build variants on cfg4/cfg3/cfg5 (each lib in its own process)
# usage: bash scripts/gpu_cmp.sh OUTDIR WORKLOADS lib...
set -o pipefail
O=gpurun_out/$1; mkdir -p $O; W=$2; shift 2
timeout -k 10 600 python -u scripts/cmp_libs.py "$W" "$@" > $O/cmp.log 2>&1
rc=$?; cat $O/cmp.log; exit $rc
