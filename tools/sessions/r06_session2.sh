#!/bin/bash
# Round 6, session 2: the pre-wake A/B again, now with spin = slices + polling inside the
# predicted arrival window (session 1's spin polled only inside it: 86 % hits), then the
# driver's command twice per candidate mode, interleaved.
set -o pipefail
O=gpurun_out/r06_s2
mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 1200 --warmup 10 --prewake-ab off,slices,spin --ab-block 10 \
  --identity-phase 0 --out $O/ab.json > $O/ab.out 2> $O/ab.err || exit $?
k=0
for arm in spin slices spin slices; do
  k=$((k + 1))
  GPUEXP_HTTP_PREWAKE=$arm timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
    --out $O/driver_${arm}_$k.json > $O/driver_${arm}_$k.out 2> $O/driver_${arm}_$k.err || exit $?
done
