#!/bin/bash
# Round 6, session 4 (last): the raw-KFD queue memory probe with the AQL rptr/wptr inputs
# (session 3 never reached it), the GPU tier on the final tree, the driver's command twice
# (median-based learnt period: the first 5 timed scrapes had lost their pre-wake), and one
# BASELINE config-5 run (100 Hz scrape + sample).
set -o pipefail
O=gpurun_out/r06_s4
mkdir -p $O
g++ -O1 tools/probe_kfd_queue.cc -I/opt/rocm/include /opt/rocm/lib/libhsakmt.a -ldrm -ldrm_amdgpu -lnuma \
  -lpthread -o $O/probe_kfd_queue > $O/probe_kfd_queue_build.txt 2>&1 || exit $?
HSAKMT_DEBUG_LEVEL=7 timeout -k 10 60 $O/probe_kfd_queue > $O/kfd_queue.txt 2>&1
rc=$?
echo "probe_kfd_queue rc=$rc" >> $O/kfd_queue.txt
rm -f $O/probe_kfd_queue
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver_$k.json \
    > $O/driver_$k.out 2> $O/driver_$k.err || exit $?
done
timeout -k 10 300 python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0 \
  --out $O/c5.json > $O/c5.out 2> $O/c5.err || exit $?
