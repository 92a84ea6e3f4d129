#!/bin/bash
# Round-4 GPU session 3 (final-tree checks): GPU tier + smoke, the driver's bench command x3
# (pre-wake from the two newest periods), BASELINE config 2 (1 Hz), config 5 (100 Hz), and
# config 1 (mock backend) on this box's CPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s3
bash tools/gpu_session.sh \
  "500::python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r04s3/pytest_gpu.log 2>&1; tail -4 gpurun_out/r04s3/pytest_gpu.log" \
  "120::python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r04s3/smoke.log 2>&1; tail -2 gpurun_out/r04s3/smoke.log" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s3/bench_driver_form_1.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s3/bench_driver_form_2.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s3/bench_driver_form_3.json" \
  "200::python -u bench.py --sample-hz 1 --scrape-hz 1 --steps 30 --warmup 3 --identity-phase 0 --out gpurun_out/r04s3/bench_config2_1hz.json" \
  "200::python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0 --out gpurun_out/r04s3/bench_config5_100hz.json" \
  "200::python -u bench.py --backend mock --steps 100 --warmup 10 --out gpurun_out/r04s3/bench_config1_mock.json"
