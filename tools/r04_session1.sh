#!/bin/bash
# Round-4 GPU session 1: SPI occupancy-limiter scope probe, read-rescue release + RSS, and the
# devices-stage A/B under the bench's GEMM pod.  Every GPU step has its own time limit; the
# first failure ends the session.
set -e
mkdir -p gpurun_out/r04
echo "[s1] spi scope $(date +%T)"
timeout -k 10 150 python -u tools/probe_spi_scope.py --seconds 2.0 > gpurun_out/r04/spi_scope.log 2>&1
grep -E "^(idle|lds_|waves_)" gpurun_out/r04/spi_scope.log || true
echo "[s1] starvation / rescue release $(date +%T)"
timeout -k 10 240 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "xcc_mfma_busy_calibration" > gpurun_out/r04/starve.log 2>&1
grep -E "starve|PASS|FAIL" gpurun_out/r04/starve.log | tail -3 || true
echo "[s1] devices A/B $(date +%T)"
tools/devices_ab.sh "${1:-2}" off duty cont late
