#!/bin/bash
# Self-sync variants side by side: bash scripts/sync_cmp.sh "cfg4 cfg2" base name ...
# (base = the default library; name = lib/libgaphuff_name.so; extra VAR=value settings
#  as name@VAR=value)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
wls=$1
shift
for spec in "$@"; do
  IFS='@' read -ra parts <<< "$spec"
  v=${parts[0]}
  if [ "$v" = base ]; then unset GAPHUFF_LIB; else export GAPHUFF_LIB=$PWD/cse375-finalproj-huffman-decoding_amd/lib/libgaphuff_$v.so; fi
  echo "== $spec"
  ( for kv in "${parts[@]:1}"; do export "$kv"; done
    timeout -k 10 300 python -u scripts/bench_sync.py $wls ) | python3 -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print("  %-5s sync_ms %.4f halo %s mism %s gaps %s bitexact %s" % (d["workload"], d["sync_ms"], d.get("halo"), d["mismatches"], d["gaps_identical"], d["bitexact"]))' || exit 1
done
