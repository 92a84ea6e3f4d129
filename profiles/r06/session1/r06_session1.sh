#!/bin/bash
# Round 6, session 1: the in-process pre-wake A/B (VERDICT r05 Next #1), then the driver's
# command with the current default and with each candidate mode.
set -o pipefail
O=gpurun_out/r06_s1
mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 1200 --warmup 10 --prewake-ab off,slices,spin --ab-block 10 \
  --identity-phase 0 --out $O/ab.json > $O/ab.out 2> $O/ab.err || exit $?
for arm in off spin slices; do
  GPUEXP_HTTP_PREWAKE=$arm timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
    --out $O/driver_$arm.json > $O/driver_$arm.out 2> $O/driver_$arm.err || exit $?
done
