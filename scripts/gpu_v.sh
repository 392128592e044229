#!/bin/bash
# Quick GPU iteration: one python process per variant (env strings such as
# "GH_MODE=tile GAPHUFF_LIB=..." apply before the library loads).  CFGS selects configs.
set -o pipefail
for c in ${CFGS:-cfg4:1000000000:0.1}; do
  for v in "$@"; do
    env $v timeout -k 10 300 python scripts/variants.py $c "$v" || exit 1
  done
done
