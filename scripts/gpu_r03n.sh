#!/bin/bash
# count kernel with a fixed store count (no vmcnt(0) per block); tile decode without the
# output-word zeroing: decode GPU tests, then timing of base vs head (HEAD~ source) on
# cfg5/cfg3 and base vs noxf (no early extra chunks) vs zero (also zeroing) vs head on cfg4, three passes each
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03n; mkdir -p $O; export TMPDIR=/tmp
step pytest 600 $O/pytest.log python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_golden_v2.py -m gpu -x -v --timeout 300 --timeout-method thread || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step cmp4 600 $O/cmp4.log python -u scripts/cmp_libs.py "cfg4:1000000000:0.1" base noxf zero head base noxf zero head base noxf zero head || exit 1
cat $O/cmp4.log
step cmp 600 $O/cmp.log python -u scripts/cmp_libs.py "cfg5:1000000000:0.5,cfg3:1000000000:0.9" base head base head || exit 1
cat $O/cmp.log
