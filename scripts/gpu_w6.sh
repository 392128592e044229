#!/bin/bash
# U=2 / 3 workgroups per CU variant: tile tests on it, then cfg4 timing vs base and prev
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/w6; mkdir -p $O; export TMPDIR=/tmp
step pyt 300 $O/pytest.log env GAPHUFF_LIB=$PWD/cse375-finalproj-huffman-decoding_amd/lib/libgaphuff_w6.so python -u -m pytest tests/test_gpu_decode.py -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread -k "tile or grouped or generated or capacity or foreign" || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u scripts/cmp_libs.py "cfg4:1000000000:0.1" base w6 prev base w6 prev
