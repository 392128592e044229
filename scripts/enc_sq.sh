#!/bin/bash
# SQ counter passes of the GPU encoder (cfg4), two separate runs
cd "$(dirname "$0")/.." 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05ak; mkdir -p $O
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
SQ2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM"
i=1
for set in "$SQ1" "$SQ2"; do
  timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/esq$i -o run -- python3 scripts/bench_encode.py cfg4 > $O/esq$i.log 2>&1 || exit 1
  python3 scripts/pmc_summary.py $O/esq$i | tee -a $O/esq.txt
  i=$((i+1))
done
