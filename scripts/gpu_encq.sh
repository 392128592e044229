#!/bin/bash
# encoder change: GPU encoder tests, then encode timings of the current and the previous build
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/encq; mkdir -p $O; export TMPDIR=/tmp
step pyt 400 $O/pytest.log python -u -m pytest tests/test_gpu_encode.py -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=$PWD/cse375-finalproj-huffman-decoding_amd/lib
step enc-base 300 $O/enc_base.log env GAPHUFF_LIB=$L/libgaphuff.so python -u scripts/bench_encode.py cfg4 cfg3 cfg2 || exit 1
cat $O/enc_base.log
step enc-prev 300 $O/enc_prev.log env GAPHUFF_LIB=$L/libgaphuff_prev.so python -u scripts/bench_encode.py cfg4 cfg3 cfg2 || exit 1
cat $O/enc_prev.log
