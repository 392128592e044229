#!/bin/bash
# SQ counter passes over quick_one.py (one workload), each pass its own run.
# WL=cfg3:1000000000:0.9 [ENVSPEC=...] bash scripts/gpu_pmc.sh "CTR CTR ..." "CTR ..."
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${R:-pmc}
mkdir -p $O
export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i+1))
  step pmc$i 120 $O/pmc$i.log env $ENVSPEC timeout -s KILL 100 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/pmc$i -o run -- python3 scripts/quick_one.py ${WL:-cfg3:1000000000:0.9} 5
  python3 scripts/pmc_summary.py $O/pmc$i
done
