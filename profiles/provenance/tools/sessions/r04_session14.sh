#!/bin/bash
# Round-4 GPU session 14: the occupancy limiters against VGPR- and SGPR-limited kernels (run
# by another process), next to the LDS- and wave-slot-limited ones.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s14
bash tools/gpu_session.sh \
  "200::python -u tools/probe_spi_scope.py --seconds 2.0 --no-self --exported --kinds lds,waves,vgpr,sgpr > gpurun_out/r04s14/spi_limiters.log 2>&1; grep -E '^(idle|lds_|waves_|vgpr_|sgpr_)' gpurun_out/r04s14/spi_limiters.log | cut -c1-330"
