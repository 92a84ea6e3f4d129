#!/bin/bash
# Round-4 GPU session 20: which runtime allocation is the exporter's 487 MiB of VRAM?  The
# queue-holding configuration under ROCr settings that move or shrink queue memory.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s20
P="python -u tools/probe_exporter_vram.py --queue-only"
bash tools/gpu_session.sh \
  "90::$P > gpurun_out/r04s20/default.log 2>&1; grep '^{' gpurun_out/r04s20/default.log | cut -c1-300" \
  "90::HSA_ALLOCATE_QUEUE_DEV_MEM=0 $P > gpurun_out/r04s20/queue_host.log 2>&1; grep '^{' gpurun_out/r04s20/queue_host.log | cut -c1-300" \
  "90::HSA_SCRATCH_MEM=0 $P > gpurun_out/r04s20/scratch0.log 2>&1; grep '^{' gpurun_out/r04s20/scratch0.log | cut -c1-300" \
  "90::HSA_ENABLE_DEBUG=0 $P > gpurun_out/r04s20/debug0.log 2>&1; grep '^{' gpurun_out/r04s20/debug0.log | cut -c1-300"
