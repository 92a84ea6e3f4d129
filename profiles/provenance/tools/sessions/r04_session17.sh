#!/bin/bash
# Round-4 GPU session 17: an 8-minute soak of the default GPU path under a GEMM pod (leaks,
# drift, counter health, scrape latency over time), tools/soak.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s17
bash tools/gpu_session.sh \
  "660::python -u tools/soak.py --minutes 8 --every 30 > gpurun_out/r04s17/soak.log 2>&1; tail -3 gpurun_out/r04s17/soak.log"
