#!/bin/bash
# Round-5 GPU session 3: config 5 (100 Hz) x3 and the driver's command x2 on the tree with the
# compiled exposition's family skipping, spliced-segment cache and settle-then-compile policy.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s3
mkdir -p $O
C5="python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0"
D="python -u bench.py --gpus 1 --steps 20 --warmup 5"
bash tools/gpu_session.sh \
  "200::$C5 --out $O/c5.1.json" "150::$D --out $O/driver.1.json" \
  "200::$C5 --out $O/c5.2.json" "150::$D --out $O/driver.2.json" \
  "200::$C5 --out $O/c5.3.json"
