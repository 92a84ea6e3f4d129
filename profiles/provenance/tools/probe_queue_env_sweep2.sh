# Second sweep of HSA runtime settings against the runtime-internal queue's 173 MiB CWSR
# area that the first user queue on a GPU brings (profiles/r02/queue_memory.txt).
set -e
mkdir -p gpurun_out/qsweep2
for v in NONE HSA_DISABLE_COREDUMP_ON_EXCEPTION=1 HSA_MAX_QUEUES=1 HSA_CO_DMACOPY_SIZE=1073741824 HSA_FORCE_SDMA_SIZE=0 HSA_ENABLE_SDMA_GANG=0 HSA_ENABLE_PEER_SDMA=0 HSA_DISCOVER_COPY_AGENTS=0 HSA_ENABLE_QUEUE_FAULT_MESSAGE=0 HSA_ENABLE_VM_FAULT_MESSAGE=0 HSA_ENABLE_SCRATCH_ALT=0 HSA_TOOLS_DISABLE_REGISTER=1; do
  if [ "$v" = NONE ]; then timeout -k 5 40 ./tools/probe_queue_mem 1 > gpurun_out/qsweep2/$v.log 2>&1; else env $v timeout -k 5 40 ./tools/probe_queue_mem 1 > gpurun_out/qsweep2/$v.log 2>&1; fi
  echo "$v: $(grep -o 'hsa_queue_create #1 (64 slots): VmRSS [0-9]* MiB' gpurun_out/qsweep2/$v.log) / destroyed $(grep -o 'queues destroyed: VmRSS [0-9]* MiB' gpurun_out/qsweep2/$v.log)" | tee -a gpurun_out/qsweep2/summary.txt
done
