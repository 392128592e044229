#!/bin/bash
# wave-tile kernel: GPU tests of the grouped paths, then cfg4 timing vs the tile kernel
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${R:-wt}
mkdir -p $O
step wttest 300 $O/wttest.log python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 120 --timeout-method thread -k "grouped_split_and_tile or wave_tile" || { tail -40 $O/wttest.log; exit 1; }
tail -5 $O/wttest.log
step q4 200 $O/q.log env GH_MODE=wtile python -u scripts/quick_one.py cfg4:1000000000:0.1 20; cat $O/q.log
step q4t 200 $O/qt.log env GH_MODE=tile python -u scripts/quick_one.py cfg4:1000000000:0.1 20; cat $O/qt.log
