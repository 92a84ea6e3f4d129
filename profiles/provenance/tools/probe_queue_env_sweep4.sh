#!/bin/bash
# ROCr's internal 64-slot compute queue appears at the first code-object load or the first
# queue creation, whichever comes first (profiles/r03/queue_memory.txt): the host->device
# copy of a code object runs on a blit-kernel queue.  Can the copy go to SDMA instead (an
# SDMA queue has no context save area)?  One probe process per setting, code object loaded
# before any queue.
set -o pipefail
P=./tools/probe_queue_mem
H=kubernetes_gpu_exporter_amd/gpuexp_sentinel.hsaco
for kv in HSA_ENABLE_SDMA=1 HSA_FORCE_SDMA_SIZE=0 HSA_FORCE_SDMA_SIZE=1 HSA_ENABLE_SDMA_COPY_SIZE_OVERRIDE=0 \
          HSA_ENABLE_SDMA_COPY_SIZE_OVERRIDE=1 HSA_ENABLE_SDMA_RECOMMENDED_ENG=0 HSA_CO_DMACOPY_SIZE=1073741824 \
          HSA_LOADER_ENABLE_MMAP_URI=1 HSA_DISCOVER_COPY_AGENTS=0; do
  echo "### $kv"
  export "$kv"
  timeout -k 5 60 $P 1 $H | grep -E "^==|queue [0-9]|queues on our"
  echo "rc=$?"
  unset "${kv%%=*}"
done
