#!/bin/bash
# wave-split change: decode tests + cfg3/cfg5/cfg2 timing vs the previous build (lib "prev")
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/wsq; mkdir -p $O; export TMPDIR=/tmp
step pyt 400 $O/pytest.log python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_golden_v2.py -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 500 python -u scripts/cmp_libs.py "cfg5:1000000000:0.5,cfg3:1000000000:0.9,cfg2:100000000:0.5" base prev base prev
