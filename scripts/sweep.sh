#!/bin/bash
# quick perf sweep over env knobs (GPU box): "PATH:U" pairs
for cfg in ${SWEEP:-"0:0"}; do
  p=${cfg%%:*}; u=${cfg##*:}
  echo "== GH_PATH=$p GH_U=$u"
  GH_PATH=$p GH_U=$u timeout -k 10 120 python scripts/quick_perf.py || exit 1
done
