#!/bin/bash
# Round-2 measurement pass: copy-bandwidth ceiling, tile-kernel skeleton, tile-kernel
# phase stamps and SQ counters on cfg4, and the slow full-size tests (cfg3/cfg4 1 GB,
# cfg5 8 GB v2).
set -o pipefail
source scripts/gpu_step.sh
O=gpurun_out/${R:-r02b}
mkdir -p $O
export TMPDIR=/tmp
step copy_bw 120 $O/copy_bw.log scripts/ubench/copy_bw; cat $O/copy_bw.log
step skel 120 $O/skel.log scripts/ubench/stream_skel; cat $O/skel.log
step stamps 300 $O/stamps.log python scripts/stamps_tile.py cfg4:1000000000:0.1; cat $O/stamps.log
step pmc-sq 120 $O/pmc_sq.log rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/pmc_sq -o run -- python3 scripts/quick_one.py cfg4:1000000000:0.1
python3 scripts/pmc_summary.py $O/pmc_sq 2>&1 | tail -20
step slow 900 $O/pytest_slow.log python -u -m pytest tests -m "gpu and slow" -q -rf --timeout 600 --timeout-method thread
tail -8 $O/pytest_slow.log
echo done
