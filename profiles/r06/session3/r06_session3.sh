#!/bin/bash
# Round 6, session 3: the final tree on silicon -- smoke(), the GPU test tier, the driver's
# command twice with the new default (pre-wake slices; per-scrape pre-wake sequence in the
# JSON), a 600-step steady-state run, one rocprofv3 kernel trace of the driver's command, and
# the raw-KFD queue memory probe with the rptr/wptr inputs (VERDICT r05 Next #6).
set -o pipefail
O=gpurun_out/r06_s3
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver_$k.json \
    > $O/driver_$k.out 2> $O/driver_$k.err || exit $?
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 600 --warmup 10 --out $O/steady600.json \
  > $O/steady600.out 2> $O/steady600.err || exit $?
export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
  -d $O/rocprof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --out $O/rocprof_bench.json \
  > $O/rocprof.log 2>&1 || exit $?
g++ -O1 tools/probe_kfd_queue.cc -I/opt/rocm/include /opt/rocm/lib/libhsakmt.a -ldrm -ldrm_amdgpu -lnuma \
  -lpthread -o $O/probe_kfd_queue > $O/probe_kfd_queue_build.txt 2>&1 || exit $?
HSAKMT_DEBUG_LEVEL=7 timeout -k 10 60 $O/probe_kfd_queue > $O/kfd_queue.txt 2>&1
rc=$?
echo "probe_kfd_queue rc=$rc" >> $O/kfd_queue.txt
rm -f $O/probe_kfd_queue
exit 0
