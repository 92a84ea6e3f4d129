#!/bin/bash
# Round 6, session 14: sessions 12 and 13 ran the driver's command right after the GPU tier and
# both saw the client's send->socket queue at 28-31 us (5-6 us in sessions 9-11).  Is that the
# box, or something the GPU tier leaves running (a process, a spinning runtime thread) that
# takes the run's CPU share?  The driver's command before and after the tier, with the cgroup's
# CPU throttling counters and a process list around it.
set -o pipefail
O=gpurun_out/r06_s14
mkdir -p $O
snap() {  # $1 = label
  { echo "== $1 $(date +%s.%N)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpu.stat 2>/dev/null
    ps -u "$(id -u)" -o pid,ppid,pcpu,etimes,nlwp,comm --sort=-pcpu; } >> $O/snapshots.txt 2>&1
}
snap start
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver_pre.json \
  > $O/driver_pre.out 2> $O/driver_pre.err || exit $?
snap after_pre
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit $?
snap after_tier
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
snap after_smoke
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out $O/driver_post.json \
  > $O/driver_post.out 2> $O/driver_post.err || exit $?
snap after_post
