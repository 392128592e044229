#!/bin/bash
# kernel time under ablations (diagnostic stamps build; outputs are wrong by design)
export GAPHUFF_LIB=$PWD/cse375-finalproj-huffman-decoding_amd/lib/libgaphuff_stamps.so
for a in 0 1 2 4 7 8 15; do
  echo "== GH_ABLATE=$a"
  GH_ABLATE=$a timeout -k 10 60 python scripts/quick_one.py cfg4:300000000:0.1 5 || exit 1
  GH_ABLATE=$a timeout -k 10 60 python scripts/quick_one.py cfg3:300000000:0.9 5 || exit 1
done
