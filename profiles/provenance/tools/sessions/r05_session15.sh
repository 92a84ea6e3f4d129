#!/bin/bash
# Round-5 GPU session 15: the final tree after the last CPU-side changes (owner change by field
# comparison, cached RCCL handles, bench problem wording): the whole GPU tier, smoke, the driver's command x2,
# config 5 x1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s15
mkdir -p $O
C5="python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0"
bash tools/gpu_session.sh \
  "700::python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1; tail -3 $O/pytest_gpu.log" \
  "180::python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1; tail -3 $O/smoke.log" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.1.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.2.json" \
  "200::$C5 --out $O/c5.1.json"
