#!/bin/bash
# PMC passes for the decode kernel on one config (run on the GPU box).
set -e
OUT=${1:-gpurun_out/pmc}
CFG=${2:-cfg4:200000000:0.1}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/$tag -o run -- python3 scripts/quick_one.py $CFG > $OUT/$tag.log 2>&1
done
