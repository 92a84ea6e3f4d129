#!/bin/bash
# Runs a sequence of GPU steps on the gpurun box, each under its own time limit.
# Test failures (exit 1) do not stop the sequence; a timeout (124/137), abort (134) or
# segfault (139) does — nothing else touches the GPU after that.
# Usage: bash tools/gpu_session.sh "<limit_s>::<cmd>" ["<limit_s>::<cmd>" ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
i=0
for spec in "$@"; do
  i=$((i + 1))
  limit="${spec%%::*}"
  cmd="${spec#*::}"
  echo "=== step $i (limit ${limit}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/step$i.log" 2>&1
  rc=$?
  echo "=== step $i rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/step$i.log"
  case $rc in
    124|137|134|139) echo "=== stopping: step $i ended with $rc" | tee -a gpurun_out/session.log; exit $rc ;;
  esac
done
exit 0
