#!/bin/bash
# encoder build variant: GPU encoder tests on it, then encode timings vs the default build
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/encv; mkdir -p $O; export TMPDIR=/tmp
L=$PWD/cse375-finalproj-huffman-decoding_amd/lib
V=${1:-e512}
step pyt 400 $O/pytest.log env GAPHUFF_LIB=$L/libgaphuff_$V.so python -u -m pytest tests/test_gpu_encode.py -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for b in base $V base $V; do
  lib=$L/libgaphuff.so; [ $b != base ] && lib=$L/libgaphuff_$b.so
  GAPHUFF_LIB=$lib step enc-$b 300 $O/enc_$b.log python -u scripts/bench_encode.py cfg4 cfg3 || exit 1
  echo "-- $b"; cut -c1-120 $O/enc_$b.log
done
