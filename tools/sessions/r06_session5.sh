#!/bin/bash
# Round 6, session 5: the CPU-side projection on an MI355X host's own CPU (wake-up charge, tick
# work warm / cold, the fake 8-GPU node at 10 / 100 Hz: the build container is an overcommitted
# VM that charges 55-110 us per wake-up), then the GPU tier, the driver's command and config 5
# on the tree with the memory reads at process_min_interval.
set -o pipefail
O=gpurun_out/r06_s5
mkdir -p $O
(lscpu; nproc; cat /proc/cmdline; grep -c processor /proc/cpuinfo) > $O/host.txt 2>&1
timeout -k 10 60 python -u tools/wakecost.py > $O/wakecost.txt 2>&1 || exit $?
timeout -k 10 240 python -u tools/tickbench.py --gpus 1,8 --hz 10,100 --ticks 1000 > $O/tickbench_warm.txt 2>&1 || exit $?
timeout -k 10 240 python -u tools/tickbench.py --gpus 8 --hz 100 --ticks 600 --sleep-ms 9 > $O/tickbench_cold100.txt 2>&1 || exit $?
timeout -k 10 240 python -u tools/tickbench.py --gpus 8 --hz 10 --ticks 150 --sleep-ms 99 > $O/tickbench_cold10.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/project_cpu.py --fetch-us 382 --policies auto --stages > $O/cpu_projection.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver_1.json \
  > $O/driver_1.out 2> $O/driver_1.err || exit $?
timeout -k 10 300 python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0 \
  --out $O/c5.json > $O/c5.out 2> $O/c5.err || exit $?
