#!/bin/bash
# quick perf sweep over env knobs (GPU box)
for sv in ${SUPERS:-1 2 4}; do
  echo "== GH_U=$sv"
  GH_U=$sv timeout -k 10 120 python scripts/quick_perf.py || exit 1
done
