#!/bin/bash
# Round 6, session 11: bench.py changed after session 10 (timed-window exposition events and
# stage means; temp dirs removed at exit).  Smoke, the driver's command, and one longer warm-up
# run for the steady-state stage means; then check that nothing of the runs is left in /tmp.
set -o pipefail
O=gpurun_out/r06_s11
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver.json \
  > $O/driver.out 2> $O/driver.err || exit $?
timeout -k 10 240 python -u bench.py --gpus 1 --steps 50 --warmup 20 --out $O/warm20.json \
  > $O/warm20.out 2> $O/warm20.err || exit $?
find /tmp -maxdepth 1 -name 'gpuexp-bench-*' | wc -l > $O/tmp_leftovers.txt  # (session 11 ran it as ls -d ... | wc -l: 0 left, but ls's no-match status made the call's rc 2)
