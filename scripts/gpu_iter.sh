#!/bin/bash
# One iteration on the GPU box: GPU tests (not slow), quick perf, optional stamps.
set -o pipefail
T=${T:-x}
timeout -k 10 400 python -m pytest tests -m "gpu and not slow" -x -q --timeout=120 > gpurun_out/t_$T.log 2>&1
rc=$?
tail -5 gpurun_out/t_$T.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/quick_perf.py > gpurun_out/p_$T.log 2>&1 || { cat gpurun_out/p_$T.log; exit 1; }
cat gpurun_out/p_$T.log
if [ -n "$STAMPS" ]; then
  timeout -k 10 200 python scripts/stamps.py $STAMPS > gpurun_out/s_$T.log 2>&1; cat gpurun_out/s_$T.log
fi
