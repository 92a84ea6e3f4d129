#!/bin/bash
# Round 6, session 13 (final tree): GPU tier + smoke + the driver's command after the counters
# budget policy moved into a pure function (counters_round_policy; same behaviour).
set -o pipefail
O=gpurun_out/r06_s13
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.json \
  > $O/driver.out 2> $O/driver.err || exit $?
find /tmp -maxdepth 1 -name 'gpuexp-bench-*' | wc -l > $O/tmp_leftovers.txt
