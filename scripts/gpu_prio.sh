#!/bin/bash
set -o pipefail
O=gpurun_out/prio; mkdir -p $O
GH_MODE=tile timeout -k 10 200 python -u scripts/cmp_libs.py cfg4:1000000000:0.1 base tp > $O/cmp.log 2>&1 || exit 1
GH_MODE=wtile timeout -k 10 200 python -u scripts/cmp_libs.py cfg4:1000000000:0.1 w8 w8p >> $O/cmp.log 2>&1 || exit 1
cat $O/cmp.log
GAPHUFF_LIB=cse375-finalproj-huffman-decoding_amd/lib/libgaphuff_s8p.so timeout -k 10 120 python -u scripts/stamps_wtile.py cfg4:1000000000:0.1
