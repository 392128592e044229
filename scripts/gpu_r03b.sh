#!/bin/bash
# round-3 evidence, part 1: GPU tests, the one-rank distributed rehearsal, the default bench line
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/r03
mkdir -p $O
export TMPDIR=/tmp
step pytest 900 $O/pytest_gpu.log python -u -m pytest tests -m "gpu and not slow" -q -rf --timeout 180 --timeout-method thread
tail -5 $O/pytest_gpu.log
step dist1 400 $O/bench_dist1.err python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --force-dist --steps 10 --warmup 3 --out-json $O/bench_dist1.json
cat $O/bench_dist1.json; tail -3 $O/bench_dist1.err
step bench-cfg4 600 $O/bench_cfg4.err python bench.py --out-json $O/bench_cfg4.json
cat $O/bench_cfg4.json
