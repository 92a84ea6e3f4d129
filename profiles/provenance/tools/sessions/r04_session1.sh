#!/bin/bash
# Round-4 GPU session 1: SPI occupancy-limiter scope probe, read-rescue release + RSS, and the
# devices-stage A/B under the bench's GEMM pod.  Each step under its own limit; a
# timeout/abort/segfault stops the session (tools/gpu_session.sh); test failures do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
bash tools/gpu_session.sh \
  "150::python -u tools/probe_spi_scope.py --seconds 2.0 > gpurun_out/r04/spi_scope.log 2>&1; grep -E '^(status|idle|lds_|waves_)' gpurun_out/r04/spi_scope.log" \
  "240::python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k xcc_mfma_busy_calibration > gpurun_out/r04/starve.log 2>&1; grep -E 'starve|passed|failed' gpurun_out/r04/starve.log | tail -3" \
  "700::tools/devices_ab.sh ${1:-2} off duty cont late"
