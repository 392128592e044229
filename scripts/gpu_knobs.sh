#!/bin/bash
# cfg4 timing of tile-kernel build/env variants (each lib in its own process), two passes
set -o pipefail
O=gpurun_out/knobs; mkdir -p $O
timeout -k 10 500 python -u scripts/cmp_libs.py "cfg4:1000000000:0.1" "$@" "$@" > $O/cmp.log 2>&1
rc=$?; cat $O/cmp.log; exit $rc
