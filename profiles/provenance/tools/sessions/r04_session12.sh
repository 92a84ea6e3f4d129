#!/bin/bash
# Round-4 GPU session 12: the full GPU tier (session 11 stopped at a feature check whose GEMM
# child had ended before the snapshot; the check now keeps it running) and smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s12
bash tools/gpu_session.sh \
  "540::python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r04s12/pytest_gpu.log 2>&1; tail -4 gpurun_out/r04s12/pytest_gpu.log" \
  "120::python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r04s12/smoke.log 2>&1; tail -2 gpurun_out/r04s12/smoke.log"
