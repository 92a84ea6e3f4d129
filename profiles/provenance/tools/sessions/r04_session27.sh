#!/bin/bash
# Round-4 GPU session 27: the counter GPU tests with the PMC read forced to the previous tick's
# end at every rate (GPUEXP_COUNTERS_KICK=end), and with the counting thread running the rounds
# (GPUEXP_PMC_INLINE=0): the non-default settings stay correct.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s27
K="counters or calibration or limiters or exporter_tick or devices_stage"
bash tools/gpu_session.sh \
  "300::GPUEXP_COUNTERS_KICK=end python -u -m pytest tests/test_gpu.py -v --timeout 240 --timeout-method thread -k '$K' > gpurun_out/r04s27/pytest_kick_end.log 2>&1; tail -2 gpurun_out/r04s27/pytest_kick_end.log" \
  "300::GPUEXP_PMC_INLINE=0 python -u -m pytest tests/test_gpu.py -v --timeout 240 --timeout-method thread -k '$K' > gpurun_out/r04s27/pytest_thread.log 2>&1; tail -2 gpurun_out/r04s27/pytest_thread.log"
