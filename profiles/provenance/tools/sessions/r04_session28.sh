#!/bin/bash
# Round-4 GPU session 28: the new 100 Hz end-kick GPU test, then the full GPU tier once more.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s28
bash tools/gpu_session.sh \
  "120::python -u -m pytest tests/test_gpu.py -v -s --timeout 120 --timeout-method thread -k 'previous_tick_end' > gpurun_out/r04s28/pytest_kick_end.log 2>&1; grep -E 'ticks,|passed|failed' gpurun_out/r04s28/pytest_kick_end.log" \
  "600::python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r04s28/pytest_gpu.log 2>&1; tail -2 gpurun_out/r04s28/pytest_gpu.log"
