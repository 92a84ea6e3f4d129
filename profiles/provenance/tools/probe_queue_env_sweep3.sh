#!/bin/bash
# Which step makes ROCr create its internal 64-slot compute queue (the second ~173 MiB
# context-save area on MI355X)?  And does any remaining ROCr knob stop it?
# Run on the GPU box from the repo root; one probe process per setting.
set -o pipefail
P=./tools/probe_queue_mem
H=kubernetes_gpu_exporter_amd/gpuexp_sentinel.hsaco
echo "### baseline, code object loaded before the first queue"
timeout -k 5 60 $P 1 $H || exit 1
for kv in HSA_CO_DMACOPY_SIZE=1073741824 HSA_ENABLE_SCRATCH_ALT=1 HSA_ENABLE_SCRATCH_ALT=0 \
          HSA_DISABLE_COREDUMP_ON_EXCEPTION=1 HSA_ENABLE_DTIF=1 HSA_ENABLE_MWAITX=1 HSA_ENABLE_SDMA_GANG=0 \
          HSA_NO_SCRATCH_THREAD_LIMITER=1 HSA_ENABLE_QUEUE_FAULT_MESSAGE=0 HSA_MAX_QUEUES=1; do
  echo "### $kv"
  export "$kv"
  timeout -k 5 60 $P 1 | grep -E "^==|queue [0-9]|queues on our" || exit 1
  unset "${kv%%=*}"
done
