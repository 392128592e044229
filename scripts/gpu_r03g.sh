#!/bin/bash
# Round-3 counters: SQ passes on the cfg4 tile kernel; FETCH_SIZE / WRITE_SIZE passes on
# cfg4, cfg3, cfg5 (each counter set its own run)
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03g; mkdir -p $O; export TMPDIR=/tmp
step sq1 120 $O/sq1.log timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/sq1 -o run -- python3 scripts/quick_one.py cfg4:1000000000:0.1 5 || exit 1
python3 scripts/pmc_summary.py $O/sq1
step sq2 120 $O/sq2.log timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM --kernel-trace --output-format csv -d $O/sq2 -o run -- python3 scripts/quick_one.py cfg4:1000000000:0.1 5 || exit 1
python3 scripts/pmc_summary.py $O/sq2
for w in cfg4 cfg3 cfg5; do
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc-$c-$w 300 $O/pmc_${c}_$w.log timeout -s KILL 280 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${c}_$w -o run -- python3 bench.py --workload $w --cpu-sample 0 --no-copy --no-e2e || exit 1
  done
done
python3 scripts/pmc_traffic.py $O/pmc_traffic.json cfg4_1000000000_n1=$O/pmc_FETCH_SIZE_cfg4,$O/pmc_WRITE_SIZE_cfg4 cfg3_1000000000_n1=$O/pmc_FETCH_SIZE_cfg3,$O/pmc_WRITE_SIZE_cfg3 cfg5_1000000000_n1=$O/pmc_FETCH_SIZE_cfg5,$O/pmc_WRITE_SIZE_cfg5 > /dev/null
cat $O/pmc_traffic.json | head -40
