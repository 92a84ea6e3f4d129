#!/bin/bash
# Round-4 GPU session 15 (final-tree checks: SGPR occupancy limiter, feature-check GEMM kept running): GPU tier +
# smoke, the driver's bench command x3, one 100-step run, and a rocprofv3 kernel trace of the
# exporter's default path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s15
bash tools/gpu_session.sh \
  "600::python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r04s15/pytest_gpu.log 2>&1; tail -4 gpurun_out/r04s15/pytest_gpu.log" \
  "120::python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r04s15/smoke.log 2>&1; tail -2 gpurun_out/r04s15/smoke.log" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s15/bench_driver_form_1.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s15/bench_driver_form_2.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s15/bench_driver_form_3.json" \
  "150::python -u bench.py --gpus 1 --steps 100 --warmup 10 --out gpurun_out/r04s15/bench_100.json" \
  "120::cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && rocprofv3 --kernel-trace --stats -d gpurun_out/r04s15/rocprof -o exporter -- python3 tools/exporter_profile.py 10 5 > gpurun_out/r04s15/rocprof.log 2>&1; tail -5 gpurun_out/r04s15/rocprof.log"
