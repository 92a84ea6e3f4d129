#!/bin/bash
# Round 6, session 9 (final tree): GPU tier + smoke, the driver's command twice, config 5, and a
# rocprofv3 kernel trace of the driver's command (partition-shared SMU fetches and the polled
# KFD event fds are in; the gpurun boxes are SPX, so the GPU tier covers that nothing changed
# for a whole GPU).
set -o pipefail
O=gpurun_out/r06_s9
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver_$k.json \
    > $O/driver_$k.out 2> $O/driver_$k.err || exit $?
done
timeout -k 10 300 python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0 \
  --out $O/c5.json > $O/c5.out 2> $O/c5.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof -o run -- python3 bench.py --gpus 1 --steps 20 \
  --warmup 5 --out $O/rocprof_bench.json > $O/rocprof.log 2>&1 || exit $?
