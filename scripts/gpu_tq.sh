#!/bin/bash
# tile-kernel change: tile tests + cfg4 timing vs the previous build (lib "prev")
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/tq; mkdir -p $O; export TMPDIR=/tmp
step pyt 300 $O/pytest.log python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_golden_v2.py -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u scripts/cmp_libs.py "cfg4:1000000000:0.1" base prev base prev base prev
