#!/bin/bash
# Round 6, session 6: the gpu tier with the new MI355X-host CPU budget tests (the fake 8-GPU
# node on the box's own CPU), smoke, and the driver's command on the tree with staggered
# RAS / detail reads.
set -o pipefail
O=gpurun_out/r06_s6
mkdir -p $O
timeout -k 10 120 python -u tools/wakecost.py > $O/wakecost.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_fakehost.py -m gpu -v -s --timeout 200 --timeout-method thread \
  -k whole_process_cpu_8_gpus_mi355x_host > $O/budget_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver_1.json \
  > $O/driver_1.out 2> $O/driver_1.err || exit $?
timeout -k 10 200 python -u tools/sigprof.py --backend amdsmi --ticks 600 --sleep-ms 99 --top 50 \
  > $O/sigprof_amdsmi_10hz.txt 2>&1 || exit $?
