#!/bin/bash
# Generic sweep: SWEEP="lib|ENV=V ENV2=V2|workload ..." entries separated by ';'
# Each entry runs quick_one.py in its own process (90 s limit); stops at the first failure.
O=gpurun_out/${R:-sweep}; mkdir -p $O
IFS=';' read -ra ENTRIES <<< "$SWEEP"
for e in "${ENTRIES[@]}"; do
  IFS='|' read -r lib envs wl <<< "$e"
  libpath=cse375-finalproj-huffman-decoding_amd/lib/libgaphuff${lib:+_$lib}.so
  echo -n "[$lib] [$envs] "
  env GAPHUFF_LIB=$libpath $envs timeout -k 10 90 python -u scripts/quick_one.py $wl ${REPS:-20} || { echo "rc=$?"; exit 1; }
done > $O/sweep.log 2>&1
cat $O/sweep.log
