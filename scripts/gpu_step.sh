#!/bin/bash
# Helpers for GPU-box scripts: run one step under its own time limit; stop the whole
# script after a fault / abort / time-limit kill (124, 134, 137, 139), carry on after
# an ordinary failure (e.g. a failing test) so the rest of the evidence still lands.
# Usage: source scripts/gpu_step.sh; step NAME SECONDS LOGFILE cmd args...
step() {
  local name=$1 secs=$2 log=$3; shift 3
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  case $rc in
    124|134|137|139) echo "!! $name ended with $rc: stopping"; tail -30 "$log"; exit $rc ;;
  esac
  return $rc
}
