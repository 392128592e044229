#!/bin/bash
# SQ counter passes (two runs) of the GPU encoder on one workload:
#   bash scripts/enc_sq.sh OUT WL [LIB]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=$1; W=$2
[ -n "$3" ] && export GAPHUFF_LIB=$PWD/cse375-finalproj-huffman-decoding_amd/lib/libgaphuff_$3.so
mkdir -p "$O"
export TMPDIR=/tmp
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
SQ2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM"
i=1
for set in "$SQ1" "$SQ2"; do
  timeout -k 10 150 timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$O/esq$i" -o run \
    -- python3 scripts/bench_encode.py "$W" > "$O/esq$i.log" 2>&1 || exit 1
  python3 scripts/pmc_summary.py "$O/esq$i" | tee -a "$O/esq.txt"
  i=$((i + 1))
done
