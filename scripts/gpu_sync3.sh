#!/bin/bash
# self-sync: the compacting walk kernel (GH_SYNC_R0 rounds per wave first; -1: old kernel)
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/sync3; mkdir -p $O; export TMPDIR=/tmp
step tests 600 $O/pytest_sync.log python -u -m pytest tests/test_sync.py -m gpu -q -x -rf --timeout 180 --timeout-method thread || { tail -30 $O/pytest_sync.log; exit 1; }
tail -3 $O/pytest_sync.log
for r in -1 1 2 3 0; do
  GH_SYNC_R0=$r step s 200 $O/s.log python -u scripts/bench_sync.py cfg4 cfg2 cfg3 || exit 1
  echo "r0=$r"; python3 -c "
import json
for l in open('$O/s.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['workload'], 'sync_ms', d['sync_ms'], 'mism', d['mismatches'], 'passes', d['passes'], 'ok', d.get('gaps_equal', d.get('gaps_ok')), d.get('bitexact'))"
done
