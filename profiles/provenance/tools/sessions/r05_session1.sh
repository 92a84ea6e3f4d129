#!/bin/bash
# Round-5 GPU session 1: the refactored PMC plugin (read machine behind ReadPort) through the
# whole GPU tier, smoke, and one driver-form bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05s1
bash tools/gpu_session.sh \
  "700::python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r05s1/pytest_gpu.log 2>&1; tail -3 gpurun_out/r05s1/pytest_gpu.log" \
  "180::python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r05s1/smoke.log 2>&1; tail -3 gpurun_out/r05s1/smoke.log" \
  "240::python -u bench.py > gpurun_out/r05s1/bench.json 2> gpurun_out/r05s1/bench.err; tail -c 1500 gpurun_out/r05s1/bench.json"
