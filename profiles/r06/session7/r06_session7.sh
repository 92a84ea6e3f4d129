#!/bin/bash
# Round 6, session 7: the tree with tick leveling, render_when_due and 1 s self histograms --
# GPU tier (incl. the MI355X-host CPU budgets), smoke, the driver's command twice, config 5,
# and the fake 8-GPU projection on this host's CPU (also with a 1 Hz scraper, render_when_due
# on / off).
set -o pipefail
O=gpurun_out/r06_s7
mkdir -p $O
timeout -k 10 120 python -u tools/wakecost.py > $O/wakecost.txt 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver_$k.json \
    > $O/driver_$k.out 2> $O/driver_$k.err || exit $?
done
timeout -k 10 300 python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0 \
  --out $O/c5.json > $O/c5.out 2> $O/c5.err || exit $?
timeout -k 10 400 python -u tools/project_cpu.py --fetch-us 382 --policies auto --stages --hz 10,100 --gpus 1,8 \
  > $O/cpu_projection.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/project_cpu.py --fetch-us 382 --policies auto --stages --hz 10 --gpus 1,8 \
  --scrape gzip --scrape-hz 1 --render-when-due 1,0 --seconds 6 > $O/render_when_due.txt 2>&1 || exit $?
