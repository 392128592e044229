#!/bin/bash
# Round GPU evidence on one MI355X: GPU tests, smoke(), bench lines (cfg2 default with
# the CPU baseline, cfg3/cfg4 without), rocprofv3 kernel-trace stats of each bench
# command, separate FETCH_SIZE / WRITE_SIZE PMC passes of each, and the per-decode
# HBM traffic derived from them (gpurun_out/$R/pmc_traffic.json); then the GPU encoder's
# numbers (scripts/bench_encode.py) and its rocprofv3 stats on cfg4.
# Usage (from the repo root, on the box): R=r01 bash scripts/round_gpu.sh
set -o pipefail
R=${R:-r01}
O=gpurun_out/$R
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -m pytest tests -m "gpu and not slow" -x -q --timeout=180 > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
step bench-cfg2
timeout -k 10 600 python bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail $O/bench_cfg2.err; exit 1; }
cat $O/bench_cfg2.json
for w in cfg3 cfg4; do
  step bench-$w
  timeout -k 10 600 python bench.py --workload $w --cpu-sample 0 > $O/bench_$w.json 2> $O/bench_$w.err \
    || { tail $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
done
TR=""
for w in cfg2 cfg3 cfg4; do
  step rocprof-stats-$w
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run \
    -- python3 bench.py --workload $w --cpu-sample 0 > $O/prof_$w.log 2>&1 || { tail $O/prof_$w.log; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc-$c-$w
    timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${c}_$w -o run \
      -- python3 bench.py --workload $w --cpu-sample 0 > $O/pmc_${c}_$w.log 2>&1 || { tail $O/pmc_${c}_$w.log; exit 1; }
  done
  TR="$TR $w=$O/pmc_FETCH_SIZE_$w,$O/pmc_WRITE_SIZE_$w"
done
python3 scripts/pmc_traffic.py $O/pmc_traffic.json $TR > /dev/null && cat $O/pmc_traffic.json
step encoder
timeout -k 10 300 python scripts/bench_encode.py > $O/encode.jsonl 2> $O/encode.err || { tail $O/encode.err; exit 1; }
cat $O/encode.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_encode -o run \
  -- python3 scripts/bench_encode.py cfg4 > $O/prof_encode.log 2>&1 || { tail $O/prof_encode.log; exit 1; }
step done
