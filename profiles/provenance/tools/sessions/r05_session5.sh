#!/bin/bash
# Round-5 GPU session 5: why the exposition is laid out again on silicon (the driver's command
# with GPUEXP_DEBUG_RELAYOUT=1), the PMC counter tests after the window-timing fix, and the
# driver's command once more.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s5
mkdir -p $O
bash tools/gpu_session.sh \
  "150::GPUEXP_DEBUG_RELAYOUT=1 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver_debug.json; cp gpurun_out/bench_exporter.log $O/exporter_relayout.log" \
  "400::python -u -m pytest tests/test_gpu.py -v --timeout 240 --timeout-method thread -k 'counters or calibration or limiters or exporter_tick or devices_stage' > $O/pytest_pmc.log 2>&1; tail -3 $O/pytest_pmc.log" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.json"
