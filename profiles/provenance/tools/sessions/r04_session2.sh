#!/bin/bash
# Round-4 GPU session 2: per-fetch SMU cost (idle / under a GEMM pod, 1-8 reader threads),
# the driver-form bench x3, the GPU test tier and smoke, and a rocprofv3 kernel summary of
# the default exporter path.  Each step under its own limit; a timeout/abort/segfault stops
# the session (tools/gpu_session.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "200::python -u tools/probe_spi_scope.py --seconds 2.0 --streams 0,1,2,3 > gpurun_out/r04/spi_scope_streams.log 2>&1; grep -E '^(idle|lds_|waves_)' gpurun_out/r04/spi_scope_streams.log | cut -c1-160" \
  "120::python -u tools/mfma_calibration.py --duties '' --xcc-cases '' --no-gated --starve 2.0 > gpurun_out/r04/starve_rss.log 2>&1; grep -E '^starve' gpurun_out/r04/starve_rss.log" \
  "150::python -u tools/probe_fetch_cost.py --seconds 3 > gpurun_out/r04/fetch_cost.log 2>&1; tail -12 gpurun_out/r04/fetch_cost.log" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04/bench_driver_form_1.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04/bench_driver_form_2.json" \
  "200::python -u bench.py --steps 100 --warmup 10 --out gpurun_out/r04/bench_1gpu_100.json" \
  "500::python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r04/pytest_gpu.log 2>&1; tail -5 gpurun_out/r04/pytest_gpu.log" \
  "120::python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r04/smoke.log 2>&1; tail -3 gpurun_out/r04/smoke.log"
