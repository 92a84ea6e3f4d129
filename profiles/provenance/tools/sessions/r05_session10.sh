#!/bin/bash
# Round-5 GPU session 10: settle after 3 stable ticks (the pod-attribution relayout's real
# parse and code build now land in the bench's warm-up, not its timed window): smoke, the
# driver's command x3, config 5 x1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s10
mkdir -p $O
C5="python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0"
bash tools/gpu_session.sh \
  "180::python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1; tail -3 $O/smoke.log" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.1.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.2.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.3.json" \
  "200::$C5 --out $O/c5.1.json"
