#!/bin/bash
# Round-4 GPU session 18: after the KFD reader's re-probe of missing GPUs -- the process and
# attribution GPU tests, smoke, and the driver's bench command twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s18
bash tools/gpu_session.sh \
  "300::python -u -m pytest tests/test_gpu.py -v --timeout 240 --timeout-method thread -k 'process or pods or exporter_tick or rccl_tracer_through or pod_energy' > gpurun_out/r04s18/pytest_procs.log 2>&1; tail -4 gpurun_out/r04s18/pytest_procs.log" \
  "120::python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r04s18/smoke.log 2>&1; tail -2 gpurun_out/r04s18/smoke.log" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s18/bench_driver_form_1.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s18/bench_driver_form_2.json"
