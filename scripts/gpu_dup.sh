#!/bin/bash
# Decode tests, cfg4 / cfg3 / cfg2 bench lines and WRITE_SIZE passes after a copy-out change.
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${R:-dup}
mkdir -p $O
export TMPDIR=/tmp
step pytest 400 $O/pytest.log python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_golden_v2.py -m gpu -q -x --timeout 180 --timeout-method thread || exit 1
tail -2 $O/pytest.log
for w in cfg4 cfg3 cfg2; do
  step bench-$w 300 $O/b_$w.err python bench.py --workload $w --cpu-sample 0 --no-copy --out-json $O/b_$w.json || exit 1
  cat $O/b_$w.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["config"]["workload"], d["ms_per_step"], d["roofline"]["achieved"], d.get("kernel_ms"))'
done
for w in cfg4 cfg3; do
  step pmc-$w 200 $O/pmc_$w.log rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmcw_$w -o run -- python3 bench.py --workload $w --cpu-sample 0 --no-copy --steps 5 --warmup 2 || exit 1
done
echo done
