#!/bin/bash
# copy-out LDS reads batched behind one wait (batch) vs one wait per read (nobatch) on cfg4;
# round-3 evidence after the scan move: full GPU suite (slow tests included), smoke, cfg4
# traffic (FETCH_SIZE / WRITE_SIZE passes, merged into profiles/pmc_traffic.json before the
# bench reads it), cfg4 bench line, kernel stats, one-rank RCCL rehearsal
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03o; mkdir -p $O; export TMPDIR=/tmp
step cmp4 600 $O/cmp4.log python -u scripts/cmp_libs.py "cfg4:1000000000:0.1" batch nobatch batch nobatch batch nobatch batch nobatch || exit 1
cat $O/cmp4.log
step pytest 900 $O/pytest.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step smoke 300 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc-$c 300 $O/pmc_$c.log timeout -s KILL 280 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${c}_cfg4 -o run -- python3 bench.py --workload cfg4 --cpu-sample 0 --no-copy --no-e2e || exit 1
done
cp profiles/pmc_traffic.json $O/pmc_traffic.json
python3 scripts/pmc_traffic.py $O/pmc_traffic.json cfg4_1000000000_n1=$O/pmc_FETCH_SIZE_cfg4,$O/pmc_WRITE_SIZE_cfg4 > /dev/null && cp $O/pmc_traffic.json profiles/pmc_traffic.json
python3 -c "import json; print(json.load(open('$O/pmc_traffic.json'))['cfg4_1000000000_n1'])"
step bench-cfg4 600 $O/bench_cfg4.err python bench.py --out-json $O/bench_cfg4.json || exit 1
cat $O/bench_cfg4.json
step prof-cfg4 400 $O/prof_cfg4.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg4 -o run -- python3 bench.py --workload cfg4 --cpu-sample 0 --no-copy --no-e2e || exit 1
step dist1 400 $O/bench_dist1.err python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --force-dist --steps 10 --warmup 3 --out-json $O/bench_dist1.json || exit 1
find $O -name "*kernel_stats.csv" | sort | while read f; do echo "== $f"; cut -d, -f1-6 "$f" | head -5; done
echo done
