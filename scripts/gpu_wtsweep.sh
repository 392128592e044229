#!/bin/bash
# wave-tile variants (libs built by `make variant V=...`) on one workload, then the tile kernel
set -o pipefail
O=gpurun_out/${R:-wtsweep}; mkdir -p $O
W=${WL:-cfg4:1000000000:0.1}
GH_MODE=${MODE:-wtile} timeout -k 10 500 python -u scripts/cmp_libs.py "$W" base ${LIBS} > $O/cmp.log 2>&1
rc=$?
GH_MODE=tile timeout -k 10 100 python -u scripts/cmp_libs.py "$W" base >> $O/cmp.log 2>&1
cat $O/cmp.log
exit $rc
