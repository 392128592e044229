#!/bin/bash
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/wt3; mkdir -p $O
step wttest 300 $O/wttest.log env GH_MODE=wtile python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread -k "grouped_split_and_tile or wave_tile or generated_vs_oracle or lut_widths or shards or capacity" || { tail -40 $O/wttest.log; exit 1; }
tail -3 $O/wttest.log
LIBS="${LIBS}" R=wt3 bash scripts/gpu_wtsweep.sh
step stamps 200 $O/stamps.log python -u scripts/stamps_wtile.py cfg4:1000000000:0.1; cat $O/stamps.log
