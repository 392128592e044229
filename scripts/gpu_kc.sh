#!/bin/bash
# Count-LUT width sweep (GH_WS_KC) on cfg3 / cfg2 / cfg5-per-GPU, then the decode tests.
source scripts/gpu_step.sh
O=gpurun_out/kc; mkdir -p $O
for kc in 0 11 12 13 14; do
  for wl in cfg3:1000000000:0.9 cfg2:100000000:0.5 cfg5:1000000000:0.5; do
    if [ $kc = 0 ]; then unset GH_WS_KC; else export GH_WS_KC=$kc; fi
    echo -n "kc=$kc "
    timeout -k 10 90 python -u scripts/quick_one.py $wl 20 || exit 1
  done
done > $O/sweep.log 2>&1
unset GH_WS_KC
step pytest 400 $O/pytest.log python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_golden_v2.py -m gpu -q -x --timeout 180 --timeout-method thread
tail -3 $O/pytest.log
