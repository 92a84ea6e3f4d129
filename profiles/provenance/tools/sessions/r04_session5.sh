#!/bin/bash
# Round-4 GPU session 5: where the exporter's CPU goes per thread on a real box, what one
# sleep/wake-up costs there, and the exposition body the driver's scrape receives.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s5
bash tools/gpu_session.sh \
  "60::python -u tools/probe_wakeup_cost.py --seconds 3 > gpurun_out/r04s5/wakeup_cost.log 2>&1; cat gpurun_out/r04s5/wakeup_cost.log" \
  "150::GPUEXP_BENCH_DUMP_EXPOSITION=gpurun_out/r04s5/exposition.txt python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s5/bench_driver_form_1.json" \
  "150::python -u bench.py --gpus 1 --steps 100 --warmup 10 --out gpurun_out/r04s5/bench_100.json"
