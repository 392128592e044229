#!/bin/bash
# PMC passes (SQ issue/wait/LDS counters, HBM bytes) of the decode kernels for the given
# configs, each counter set in its own rocprofv3 pass.  Run on the GPU box from the repo root.
# Usage: TAG=x bash scripts/prof_counters.sh cfg4:1000000000:0.1 cfg3:1000000000:0.9
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc${TAG}
mkdir -p $O
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM"
      "FETCH_SIZE" "WRITE_SIZE")
for c in "$@"; do
  n=$(echo $c | cut -d: -f1)
  i=0; mkdir -p $O/$n
  for set in "${SETS[@]}"; do
    timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/$n/p$i -o run \
      -- python3 scripts/quick_one.py $c 3 > $O/$n/p$i.log 2>&1 || { tail -5 $O/$n/p$i.log; exit 1; }
    i=$((i+1))
  done
  echo "=== $n"; python3 scripts/pmc_summary.py $O/$n
done
