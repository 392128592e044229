#!/bin/bash
# tile kernel: window-word trimming + wave scans before the copy-out; decode GPU tests on
# the new default lib, then cfg4 timing of base / notrim / head (HEAD source) x3 passes
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03m; mkdir -p $O; export TMPDIR=/tmp
step pytest 600 $O/pytest.log python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_golden_v2.py -m gpu -x -v --timeout 300 --timeout-method thread || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step cmp 600 $O/cmp.log python -u scripts/cmp_libs.py "cfg4:1000000000:0.1" base notrim head base notrim head base notrim head || exit 1
cat $O/cmp.log
