#!/bin/bash
# long-code streams: wave split vs the round-2 multi split, kernel stats per structure
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/lc; mkdir -p $O
export TMPDIR=/tmp
step ws 300 $O/ws.txt rocprofv3 --kernel-trace --stats -d $O/ws -o ws -- python3 -u scripts/time_longcodes.py --n 1000000000
cat $O/ws.txt


find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-4 "$f" | head -8; done
