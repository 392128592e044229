set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/wt2; mkdir -p $O
step wttest 300 $O/wttest.log env GH_MODE=wtile python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread -k "grouped_split_and_tile or wave_tile or generated_vs_oracle or lut_widths or shards" || { tail -40 $O/wttest.log; exit 1; }
tail -3 $O/wttest.log
LIBS="pf1 pf2a1 pf2a3" R=wt2 bash scripts/gpu_wtsweep.sh
