#!/bin/bash
# Round-4 GPU session 19: the exporter's own VRAM footprint per GPU source (idle GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s19
bash tools/gpu_session.sh \
  "200::python -u tools/probe_exporter_vram.py > gpurun_out/r04s19/exporter_vram.log 2>&1; cat gpurun_out/r04s19/exporter_vram.log | cut -c1-300"
