#!/bin/bash
# self-sync walk: lock-step round cap sweep (GH_SYNC_ROUNDS) x halo on cfg4/cfg2/cfg3
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/syncsw; mkdir -p $O; export TMPDIR=/tmp
for h in 8 16; do for r in 0 1 2 3 5; do
  GH_SYNC_HALO=$h GH_SYNC_ROUNDS=$r step s$h-$r 200 $O/s_${h}_$r.log python -u scripts/bench_sync.py cfg4 cfg2 cfg3 || exit 1
  echo "halo=$h rounds=$r"; cut -c1-300 $O/s_${h}_$r.log
done; done
