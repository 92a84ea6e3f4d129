set -e
mkdir -p gpurun_out/r02h
for v in NONE HSA_DISABLE_PC_SAMPLING=1 HSA_ALLOCATE_QUEUE_DEV_MEM=1 HSA_NO_SCRATCH_RECLAIM=1 HSA_ENABLE_SCRATCH_ASYNC_RECLAIM=0 HSA_CU_MASK_SKIP_INIT=1 HSA_ENABLE_DEBUG=0 HSA_DISABLE_CACHE=1 HSA_SCRATCH_MEM=0 HSA_ENABLE_INTERRUPT=0; do
  if [ "$v" = NONE ]; then timeout -k 5 40 ./tools/probe_queue_mem 1 > gpurun_out/r02h/$v.log 2>&1; else env $v timeout -k 5 40 ./tools/probe_queue_mem 1 > gpurun_out/r02h/$v.log 2>&1; fi
  echo "$v: $(grep -o 'hsa_queue_create #1 (64 slots): VmRSS [0-9]* MiB' gpurun_out/r02h/$v.log) / destroyed $(grep -o 'queues destroyed: VmRSS [0-9]* MiB' gpurun_out/r02h/$v.log)" >> gpurun_out/r02h/summary.txt
done
