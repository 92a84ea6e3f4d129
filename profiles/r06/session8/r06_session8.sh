#!/bin/bash
# Round 6, session 8: the tree with render_when_due skipping the table writes too.  GPU tier +
# smoke, the driver's command, a Prometheus-like 1 Hz scraper against the 10 Hz sampler with
# render_when_due on / off (interleaved x2), BASELINE config 2 (1 Hz), and a 5-minute soak.
set -o pipefail
O=gpurun_out/r06_s8
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver_1.json \
  > $O/driver_1.out 2> $O/driver_1.err || exit $?
for k in 1 2; do
  for rwd in 1 0; do
    GPUEXP_RENDER_WHEN_DUE=$rwd timeout -k 10 200 python -u bench.py --sample-hz 10 --scrape-hz 1 --steps 30 \
      --warmup 3 --identity-phase 0 --out $O/scrape1hz_rwd${rwd}_$k.json > $O/scrape1hz_rwd${rwd}_$k.out \
      2> $O/scrape1hz_rwd${rwd}_$k.err || exit $?
  done
done
timeout -k 10 200 python -u bench.py --sample-hz 1 --scrape-hz 1 --steps 30 --warmup 3 --identity-phase 0 \
  --out $O/config2_1hz.json > $O/config2_1hz.out 2> $O/config2_1hz.err || exit $?
timeout -k 10 420 python -u tools/soak.py --minutes 5 --every 30 > $O/soak.txt 2>&1 || exit $?
