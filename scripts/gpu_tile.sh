#!/bin/bash
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${R:-tile}
mkdir -p $O
step tiletest 400 $O/tiletest.log python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_io.py tests/test_gpu_golden_v2.py -q -x --timeout 120 --timeout-method thread; tail -4 $O/tiletest.log
step cmp 600 $O/cmp.log python scripts/cmp_libs.py "${WL:-cfg4:1000000000:0.1}" ${LIBS:-base}; cat $O/cmp.log
