#!/bin/bash
# wave-tile stamps at several count-ahead distances (libs libgaphuff_sL.so)
set -o pipefail
O=gpurun_out/wtL; mkdir -p $O
for L in ${LS:-2 4 6 8}; do
  GAPHUFF_LIB=cse375-finalproj-huffman-decoding_amd/lib/libgaphuff_s$L.so timeout -k 10 120 python -u scripts/stamps_wtile.py cfg4:1000000000:0.1 > $O/s$L.log 2>&1 || { cat $O/s$L.log; exit 1; }
  echo "== L=$L"; head -3 $O/s$L.log
done
