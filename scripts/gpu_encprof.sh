#!/bin/bash
# encoder kernels' times (rocprofv3 kernel stats), current vs previous build, cfg4
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/encprof; mkdir -p $O; export TMPDIR=/tmp
L=$PWD/cse375-finalproj-huffman-decoding_amd/lib
for b in base prev; do
  lib=$L/libgaphuff.so; [ $b = prev ] && lib=$L/libgaphuff_prev.so
  GAPHUFF_LIB=$lib step prof-$b 300 $O/prof_$b.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$b -o run -- python3 scripts/bench_encode.py cfg4 || exit 1
  echo "== $b"; cut -d, -f1-4 $O/prof_$b/run_kernel_stats.csv | head -8
done
