#!/bin/bash
# Round 6, session 15 (final tree): GPU tier + smoke + the driver's command, and the CPX
# projection on the host's CPU, after PMC round leveling.  A round stretched by
# counters_cpu_budget is put off one tick from a predicted two-fetch tick.  A stretched round
# weighs as two fetches in the extras' leveling.  Both are inactive at one or eight whole GPUs.
set -o pipefail
O=gpurun_out/r06_s15
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.json \
  > $O/driver.out 2> $O/driver.err || exit $?
for b in 0 0.75; do
  timeout -k 10 120 python -u tools/project_cpx.py --counters-budget $b > $O/cpx_budget_$b.txt 2> $O/cpx_budget_$b.err || exit $?
done
