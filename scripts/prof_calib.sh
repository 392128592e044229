#!/bin/bash
# LDS/VALU counter calibration: ubench lds_chain (known LDS-bound configs) and the
# decoder on cfg4 (300 MB) with the same counter sets; also lists counters.
set -o pipefail
OUT=gpurun_out/calib
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for set in "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -k 10 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/ub_$tag -o run -- scripts/ubench/lds_chain > $OUT/ub_$tag.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/dec_$tag -o run -- python3 scripts/quick_one.py cfg4:300000000:0.1 > $OUT/dec_$tag.log 2>&1 || exit 1
done
