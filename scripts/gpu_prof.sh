#!/bin/bash
# Kernel-level breakdown: rocprofv3 --kernel-trace --stats of quick_one.py per workload.
# WL="cfg3:1000000000:0.9,cfg5:..." [ENVSPEC="GH_MODE=msplit"] bash scripts/gpu_prof.sh
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${R:-prof}
mkdir -p $O
export TMPDIR=/tmp
IFS=',' read -ra W <<< "${WL:-cfg3:1000000000:0.9}"
for wl in "${W[@]}"; do
  n=${wl%%:*}
  step prof-$n 300 $O/prof_$n.log env $ENVSPEC rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- python3 scripts/quick_one.py $wl 20
  grep -h "ms=" $O/prof_$n.log
  find $O/prof_$n -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \; | grep -v rocclr
done
