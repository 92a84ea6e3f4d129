#!/bin/bash
# Round 6, session 10 (final tree): GPU tier + smoke, the driver's command twice, and the CPX
# projection (tools/project_cpx.py) on the MI355X host's CPU.  New since session 9: PMC read
# rounds under counters_cpu_budget (no change at one whole GPU: a round is ~15 us), amdsmi
# partitions grouped by socket handle.
set -o pipefail
O=gpurun_out/r06_s10
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver_$k.json \
    > $O/driver_$k.out 2> $O/driver_$k.err || exit $?
done
for b in 0 0.75; do
  timeout -k 10 120 python -u tools/project_cpx.py --counters-budget $b > $O/cpx_budget_$b.txt 2> $O/cpx_budget_$b.err || exit $?
done
