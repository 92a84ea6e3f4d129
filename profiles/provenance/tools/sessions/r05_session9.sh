#!/bin/bash
# Round-5 GPU session 9: the whole GPU tier again (session 8's new silicon exposition test
# scraped before the first tick; it now waits for readiness), smoke, the driver's command x2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s9
mkdir -p $O
bash tools/gpu_session.sh \
  "700::python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1; tail -3 $O/pytest_gpu.log" \
  "180::python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1; tail -3 $O/smoke.log" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.1.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.2.json"
