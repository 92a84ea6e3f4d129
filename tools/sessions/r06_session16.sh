#!/bin/bash
# Round 6, session 16: BASELINE config 5 (100 Hz scrape + sample, 1000 timed scrapes) on the
# final tree (last measured in session 9, before counters_cpu_budget and round leveling; at one
# GPU neither is active, so this checks that nothing else moved).
set -o pipefail
O=gpurun_out/r06_s16
mkdir -p $O
timeout -k 10 300 python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0 \
  --out $O/c5.json > $O/c5.out 2> $O/c5.err || exit $?
