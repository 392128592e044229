#!/bin/bash
# One GPU lease, parameterised (replaces the per-experiment gpu_*.sh wrappers).
#
#   gpurun -- bash scripts/lease.sh OUT STEP [STEP ...]
#
# OUT is a directory under gpurun_out/.  Each STEP is one quoted argument:
#   tests                     pytest -m "gpu and not slow"
#   slow                      pytest -m "gpu and slow"
#   smoke                     __graft_entry__.smoke()
#   perf WL...                quick_one.py per workload (kernel ms, frac, bit-exact)
#   cmp WL[,WL] LIB...        cmp_libs.py: build variants side by side (LIB = base | name[@VAR=v...])
#   cmpss WL[,WL] LIB...      the same in the steady state (60 untimed + 100 timed decodes each)
#   bench NAME [ARGS...]      bench.py ARGS --out-json OUT/NAME.json
#   stats NAME WL             rocprofv3 --kernel-trace --stats of quick_one.py WL
#   sq NAME WL [LIB]          two SQ counter passes (issue / wait / LDS) of quick_one.py WL
#                             (LIB: a build variant's name, lib/libgaphuff_LIB.so)
#   traffic NAME WL [V=x]     FETCH_SIZE and WRITE_SIZE passes (separate runs), with settings
#   cmd NAME SECS CMD...      anything else, under its own time limit
# WL: cfg2 | cfg3 | cfg4 | cfg5 | name:N:r.  Every step runs under its own `timeout -k`;
# a fault / abort / time-limit kill (124, 134, 137, 139) ends the lease (gpu_step.sh),
# an ordinary failure (a failing test) does not.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
source scripts/gpu_step.sh
O=$1
shift
mkdir -p "$O"
export TMPDIR=/tmp

wl() {
  case $1 in
    cfg2) echo cfg2:100000000:0.5 ;;
    cfg3) echo cfg3:1000000000:0.9 ;;
    cfg4) echo cfg4:1000000000:0.1 ;;
    cfg5) echo cfg5:1000000000:0.5 ;;
    *) echo "$1" ;;
  esac
}

SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
SQ2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM"

for spec in "$@"; do
  read -ra a <<< "$spec"
  kind=${a[0]}
  case $kind in
    tests)
      step tests 900 "$O/tests.log" python -u -m pytest tests -m "gpu and not slow" -q -rf -x \
        --timeout 180 --timeout-method thread || true
      tail -4 "$O/tests.log" ;;
    slow)
      step slow 900 "$O/slow.log" python -u -m pytest tests -m "gpu and slow" -v -rf \
        --timeout 600 --timeout-method thread --durations=0 || true
      tail -12 "$O/slow.log" ;;
    smoke)
      step smoke 300 "$O/smoke.log" python -c "import __graft_entry__ as g; g.smoke()" || true
      cat "$O/smoke.log" ;;
    perf)
      for w in "${a[@]:1}"; do
        step "perf-$w" 300 "$O/perf_$w.log" python -u scripts/quick_one.py "$(wl "$w")" 20 || true
        cat "$O/perf_$w.log"
      done ;;
    cmp|cmpss)
      if [ "$kind" = cmpss ]; then export QO_WARM=60 CMP_REPS=100; fi
      ws=""
      IFS=',' read -ra wls <<< "${a[1]}"
      for w in "${wls[@]}"; do ws="$ws${ws:+,}$(wl "$w")"; done
      step "$kind" 900 "$O/${kind}_${a[1]//,/_}.log" python -u scripts/cmp_libs.py "$ws" "${a[@]:2}" || true
      unset QO_WARM CMP_REPS
      cat "$O/${kind}_${a[1]//,/_}.log" ;;
    bench)
      step "bench-${a[1]}" 600 "$O/bench_${a[1]}.err" python bench.py "${a[@]:2}" --out-json "$O/${a[1]}.json" || true
      cat "$O/${a[1]}.json" 2> /dev/null || tail -20 "$O/bench_${a[1]}.err" ;;
    stats)
      step "stats-${a[1]}" 400 "$O/stats_${a[1]}.log" rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$O/stats_${a[1]}" -o run -- python3 scripts/quick_one.py "$(wl "${a[2]}")" 20 || true
      f=$(find "$O/stats_${a[1]}" -name '*kernel_stats.csv' | head -1)
      [ -n "$f" ] && cp "$f" "$O/${a[1]}_kernel_stats.csv" && cat "$O/${a[1]}_kernel_stats.csv" ;;
    sq)
      if [ -n "${a[3]}" ]; then export GAPHUFF_LIB=$PWD/cse375-finalproj-huffman-decoding_amd/lib/libgaphuff_${a[3]}.so; fi
      i=1
      for set in "$SQ1" "$SQ2"; do
        step "sq$i-${a[1]}" 150 "$O/sq${i}_${a[1]}.log" timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace \
          --output-format csv -d "$O/sq${i}_${a[1]}" -o run -- python3 scripts/quick_one.py "$(wl "${a[2]}")" 5 || exit 1
        python3 scripts/pmc_summary.py "$O/sq${i}_${a[1]}" | tee -a "$O/sq_${a[1]}.txt"
        i=$((i + 1))
      done
      unset GAPHUFF_LIB ;;
    traffic)
      for kv in "${a[@]:3}"; do export "$kv"; done  # optional VAR=value settings (e.g. GH_MODE=mtile)
      for c in FETCH_SIZE WRITE_SIZE; do
        step "pmc-$c-${a[1]}" 150 "$O/pmc_${c}_${a[1]}.log" timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace \
          --output-format csv -d "$O/pmc_${c}_${a[1]}" -o run -- python3 scripts/quick_one.py "$(wl "${a[2]}")" 5 || exit 1
        python3 scripts/pmc_summary.py "$O/pmc_${c}_${a[1]}" | tee -a "$O/traffic_${a[1]}.txt"
      done
      for kv in "${a[@]:3}"; do unset "${kv%%=*}"; done ;;
    cmd)
      step "${a[1]}" "${a[2]}" "$O/${a[1]}.log" "${a[@]:3}" || true
      tail -40 "$O/${a[1]}.log" ;;
    *)
      echo "unknown step: $spec"; exit 2 ;;
  esac
done
echo "lease done"
