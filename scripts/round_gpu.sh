#!/bin/bash
# Round GPU evidence on one MI355X (R=r02 bash scripts/round_gpu.sh): GPU tests (fast
# and slow), smoke(), the default bench line (cfg4, with the CPU baselines), cfg3 / cfg2
# / cfg5 lines, rocprofv3 kernel-trace stats of each bench command, separate
# FETCH_SIZE / WRITE_SIZE PMC passes for cfg4 and cfg3 (-> pmc_traffic.json, keyed
# workload_bytes_nGPUs), the GPU encoder and self-sync numbers.
set -o pipefail
source scripts/gpu_step.sh
R=${R:-r02}
O=gpurun_out/$R
mkdir -p $O
export TMPDIR=/tmp
step pytest 900 $O/pytest_gpu.log python -u -m pytest tests -m "gpu and not slow" -q -rf --timeout 180 --timeout-method thread
tail -4 $O/pytest_gpu.log
step pytest-slow 900 $O/pytest_slow.log python -u -m pytest tests -m "gpu and slow" -v -rf --timeout 600 --timeout-method thread --durations=0
tail -12 $O/pytest_slow.log
step smoke 300 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()"; cat $O/smoke.log
step bench-cfg4 600 $O/bench_cfg4.err python bench.py --out-json $O/bench_cfg4.json; cat $O/bench_cfg4.json
for w in cfg3 cfg2 cfg5; do
  step bench-$w 400 $O/bench_$w.err python bench.py --workload $w --cpu-sample 0 --out-json $O/bench_$w.json; cat $O/bench_$w.json
done
TR=""
for w in cfg4 cfg3 cfg2; do
  step rocprof-$w 400 $O/prof_$w.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py --workload $w --cpu-sample 0 --no-copy
done
for w in cfg4 cfg3; do
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc-$c-$w 300 $O/pmc_${c}_$w.log rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${c}_$w -o run -- python3 bench.py --workload $w --cpu-sample 0 --no-copy
  done
  TR="$TR ${w}_1000000000_n1=$O/pmc_FETCH_SIZE_$w,$O/pmc_WRITE_SIZE_$w"
done
python3 scripts/pmc_traffic.py $O/pmc_traffic.json $TR > /dev/null && cat $O/pmc_traffic.json
step encoder 300 $O/encode.jsonl python scripts/bench_encode.py; cat $O/encode.jsonl
step sync 300 $O/sync.jsonl python scripts/bench_sync.py; cat $O/sync.jsonl
echo done
