#!/bin/bash
# SQ counter passes on the cfg4 tile kernel (each counter set its own run)
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${1:-sq}; mkdir -p $O; export TMPDIR=/tmp
step sq1 120 $O/sq1.log timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/sq1 -o run -- python3 scripts/quick_one.py cfg4:1000000000:0.1 5 || exit 1
python3 scripts/pmc_summary.py $O/sq1
step sq2 120 $O/sq2.log timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM --kernel-trace --output-format csv -d $O/sq2 -o run -- python3 scripts/quick_one.py cfg4:1000000000:0.1 5 || exit 1
python3 scripts/pmc_summary.py $O/sq2
