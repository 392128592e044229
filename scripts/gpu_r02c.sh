#!/bin/bash
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${R:-r02c}
mkdir -p $O
export TMPDIR=/tmp
step direct 120 $O/direct.log scripts/ubench/direct_store; cat $O/direct.log
step ablate 400 $O/ablate.log python scripts/stamps_tile.py cfg4:1000000000:0.1 0 32 2 4 6 38 8 40; cat $O/ablate.log
step bench 300 $O/bench.err python bench.py --cpu-sample 0 --out-json $O/bench.json; cat $O/bench.json
echo done
