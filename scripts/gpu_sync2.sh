#!/bin/bash
# self-sync: default (1 round) tests + round/halo sweep incl. 0 rounds
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/sync2; mkdir -p $O; export TMPDIR=/tmp
step tests 600 $O/pytest_sync.log python -u -m pytest tests/test_sync.py -m gpu -q -rf --timeout 180 --timeout-method thread
tail -4 $O/pytest_sync.log
for hr in "8 1" "8 2" "16 1" "8 -1"; do set -- $hr
  GH_SYNC_HALO=$1 GH_SYNC_ROUNDS=$2 step s 200 $O/s.log python -u scripts/bench_sync.py cfg4 cfg2 cfg3 || exit 1
  echo "halo=$1 rounds=$2"; python3 -c "
import json,sys
for l in open('$O/s.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['workload'], 'sync_ms', d['sync_ms'], 'mism', d['mismatches'], 'passes', d['passes'])"
done
