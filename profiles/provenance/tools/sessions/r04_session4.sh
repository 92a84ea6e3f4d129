#!/bin/bash
# Round-4 GPU session 4: do SPI_CSN_WAVE / SPI_CSN_NUM_THREADGROUPS count other processes'
# waves on an unprivileged box (a device-wide waves/s like the occupancy limiters)?  Known
# launches: lds kernel 2048 one-wave blocks, waves kernel 4096 eight-wave blocks, per 2 s case.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s4
bash tools/gpu_session.sh \
  "200::GPUEXP_PMC_SPI_WAVES=1 python -u tools/probe_spi_scope.py --seconds 2.0 --streams 0,2 > gpurun_out/r04s4/spi_waves.log 2>&1; grep -E '^(idle|lds_|waves_)' gpurun_out/r04s4/spi_waves.log | cut -c1-400"
