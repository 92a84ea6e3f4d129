#!/bin/bash
# Round-5 GPU session 16: gpu_metrics fetch CPU against the phase of the PMFW's table refresh
# (tools/probe_fetch_phase.py), under the GEMM pod and idle.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s16
mkdir -p $O
bash tools/gpu_session.sh \
  "120::python -u tools/probe_fetch_phase.py --seconds 40 > $O/phase_loaded.txt 2>&1; tail -16 $O/phase_loaded.txt" \
  "90::python -u tools/probe_fetch_phase.py --seconds 25 --no-load > $O/phase_idle.txt 2>&1; tail -16 $O/phase_idle.txt"
