#!/bin/bash
# round-3 evidence, wave split and counters: cfg3/cfg5/cfg2 bench lines and kernel stats
# (count kernel with fixed stores), SQ passes on the cfg4 tile kernel after the scan move
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03p; mkdir -p $O; export TMPDIR=/tmp
for w in cfg3 cfg5 cfg2; do
  step bench-$w 400 $O/bench_$w.err python bench.py --workload $w --cpu-sample 0 --no-e2e --out-json $O/bench_$w.json || exit 1
  step prof-$w 400 $O/prof_$w.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py --workload $w --cpu-sample 0 --no-copy --no-e2e || exit 1
done
for w in cfg3 cfg5 cfg2; do python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', d['roofline']['kernel_ms'], d['value'], d['roofline']['frac'], d['roofline']['copy_frac'], d['bitexact'])"; done
step sq1 120 $O/sq1.log timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/sq1 -o run -- python3 scripts/quick_one.py cfg4:1000000000:0.1 5 || exit 1
python3 scripts/pmc_summary.py $O/sq1
step sq2 120 $O/sq2.log timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM --kernel-trace --output-format csv -d $O/sq2 -o run -- python3 scripts/quick_one.py cfg4:1000000000:0.1 5 || exit 1
python3 scripts/pmc_summary.py $O/sq2
find $O -name "*kernel_stats.csv" | sort | while read f; do echo "== $f"; cut -d, -f1-6 "$f" | head -5; done
echo done
