#!/bin/bash
# Round-4 GPU session 23: per-process cost of KFD process discovery and pod attribution with
# 1/4/8/12 GPU processes on one MI355X (tools/probe_many_procs.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s23
bash tools/gpu_session.sh \
  "300::python -u tools/probe_many_procs.py --counts 1,4,8,12 --seconds 3 > gpurun_out/r04s23/many_procs.log 2>&1; grep -E '^\{' gpurun_out/r04s23/many_procs.log | cut -c1-300"
