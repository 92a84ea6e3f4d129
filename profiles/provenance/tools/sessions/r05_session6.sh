#!/bin/bash
# Round-5 GPU session 6: the tree with literal-only settling, field room at first layout and the
# PMC window-timing fix: the whole GPU tier, smoke, the driver's command x2 (one with the relayout
# log), config 5 x2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s6
mkdir -p $O
C5="python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0"
bash tools/gpu_session.sh \
  "700::python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1; tail -3 $O/pytest_gpu.log" \
  "180::python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1; tail -3 $O/smoke.log" \
  "150::GPUEXP_DEBUG_RELAYOUT=1 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.1.json; cp gpurun_out/bench_exporter.log $O/exporter_relayout.log" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.2.json" \
  "200::$C5 --out $O/c5.1.json" \
  "200::$C5 --out $O/c5.2.json"
