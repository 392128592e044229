#!/bin/bash
# Encoder variants side by side: bash scripts/enc_cmp.sh "cfg4 cfg3" base name ...
# (base = the default library; name = lib/libgaphuff_name.so)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
wls=$1
shift
for v in "$@"; do
  if [ "$v" = base ]; then unset GAPHUFF_LIB; else export GAPHUFF_LIB=$PWD/cse375-finalproj-huffman-decoding_amd/lib/libgaphuff_$v.so; fi
  echo "== $v"
  timeout -k 10 200 python -u scripts/bench_encode.py $wls | python3 -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print("  %-5s encode_ms %.4f identical %s" % (d["workload"], d["encode_ms"], d["identical_to_host"]))' || exit 1
done
