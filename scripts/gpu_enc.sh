#!/bin/bash
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${R:-enc}
mkdir -p $O
step enctest 300 $O/enctest.log python -u -m pytest tests/test_gpu_encode.py -q -x --timeout 120 --timeout-method thread; tail -3 $O/enctest.log
step encnew 300 $O/encnew.log python scripts/bench_encode.py; cat $O/encnew.log
step encold 300 $O/encold.log env GAPHUFF_LIB=cse375-finalproj-huffman-decoding_amd/lib/libgaphuff_uc2.so python scripts/bench_encode.py; cat $O/encold.log
