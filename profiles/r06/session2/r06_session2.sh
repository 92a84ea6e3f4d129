#!/bin/bash
# Round 6, session 2 (VERDICT r05 Next #1, #6, #5 on silicon):
#  1. the pre-wake A/B again, now with spin = slices + polling inside the predicted arrival
#     window (session 1's spin polled only inside it: 86 % hits), then the driver's command
#     twice per candidate mode, interleaved;
#  2. the memory floor: exporter RSS per optional-source variant (tools/probe_rss.py), and one
#     compute queue created straight through KFD without ROCr (tools/probe_kfd_queue.cc);
#  3. the GPU test tier on the split engine + table-driven families.
set -o pipefail
O=gpurun_out/r06_s2
mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 1200 --warmup 10 --prewake-ab off,slices,spin --ab-block 10 \
  --identity-phase 0 --out $O/ab.json > $O/ab.out 2> $O/ab.err || exit $?
k=0
for arm in spin slices spin slices; do
  k=$((k + 1))
  GPUEXP_HTTP_PREWAKE=$arm timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
    --out $O/driver_${arm}_$k.json > $O/driver_${arm}_$k.out 2> $O/driver_${arm}_$k.err || exit $?
done
timeout -k 10 120 python -u tools/probe_rss.py > $O/exporter_rss.txt 2>&1 || exit $?
g++ -O1 tools/probe_kfd_queue.cc -I/opt/rocm/include /opt/rocm/lib/libhsakmt.a -ldrm -ldrm_amdgpu -lnuma \
  -lpthread -o $O/probe_kfd_queue > $O/probe_kfd_queue_build.txt 2>&1 || exit $?
timeout -k 10 60 $O/probe_kfd_queue > $O/kfd_queue.txt 2>&1
echo "probe_kfd_queue rc=$?" >> $O/kfd_queue.txt
rm -f $O/probe_kfd_queue
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit $?
