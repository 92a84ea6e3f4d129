#!/bin/bash
# Round-5 GPU session 4: the whole GPU tier, smoke and the driver's command x2 on the tree with
# the KFD-vouched resolver, the per-process attribution cache and pre-wake off by default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s4
mkdir -p $O
bash tools/gpu_session.sh \
  "700::python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1; tail -3 $O/pytest_gpu.log" \
  "180::python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1; tail -3 $O/smoke.log" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.1.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.2.json"
