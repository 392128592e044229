#!/bin/bash
# quick perf sweep over env knobs (GPU box)
for sv in ${SUPERS:-1 2 4 8}; do
  echo "== GH_SUPER=$sv"
  GH_SUPER=$sv timeout -k 10 120 python scripts/quick_perf.py || exit 1
done
