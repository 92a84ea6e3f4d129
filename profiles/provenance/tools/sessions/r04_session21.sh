#!/bin/bash
# Round-4 GPU session 21: BASELINE config 5 (100 Hz) with the PMC read kicked at the end of the
# previous tick (counters_kick auto) vs at the tick's start, interleaved; then the driver form
# (10 Hz: auto = start, unchanged) and the counter GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s21
B="python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0"
bash tools/gpu_session.sh \
  "200::$B --out gpurun_out/r04s21/c5_auto.1.json" \
  "200::GPUEXP_COUNTERS_KICK=start $B --out gpurun_out/r04s21/c5_start.1.json" \
  "200::$B --out gpurun_out/r04s21/c5_auto.2.json" \
  "200::GPUEXP_COUNTERS_KICK=start $B --out gpurun_out/r04s21/c5_start.2.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s21/bench_driver_form.json" \
  "300::python -u -m pytest tests/test_gpu.py -v --timeout 240 --timeout-method thread -k 'counters or calibration or limiters or exporter_tick or devices_stage' > gpurun_out/r04s21/pytest_pmc.log 2>&1; tail -3 gpurun_out/r04s21/pytest_pmc.log"
