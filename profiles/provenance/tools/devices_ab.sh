#!/bin/bash
# Devices-stage A/B under the bench's GEMM pod (VERDICT r03 "do this" #1): which part of the
# exporter's devices stage grew from round 2 (177 us) to round 3 (500 us), and what fixes it.
# Arms, interleaved, REPS rounds (each arm = one short bench.py run on the same box):
#   off        no PMC counters, no sentinel (no exporter GPU queue)
#   duty       PMC counters, 20 ms windows
#   cont       continuous PMC, read kicked at the tick's start (round-3 default)
#   late       continuous PMC, read kicked after the gpu_metrics SMU fetch
#   r02        round-2 HEAD's exporter (ab_r02 worktree) under this tree's bench workload
# Usage: tools/devices_ab.sh REPS ARMS...   (results: gpurun_out/ab/<arm>.<rep>.json)
set -e
reps=${1:-3}; shift
arms=${*:-off duty cont late}
mkdir -p gpurun_out/ab
for rep in $(seq 1 "$reps"); do
  for arm in $arms; do
    extra=(); envs=()
    case $arm in
      off) extra=(--counters 0 --sentinel 0) ;;  # no exporter GPU queue at all (flagged degraded: rc 1)
      duty) envs=(GPUEXP_COUNTERS_MODE=duty) ;;
      cont) envs=(GPUEXP_COUNTERS_KICK=start) ;;
      late) envs=(GPUEXP_COUNTERS_KICK=after_devices) ;;
      r02) envs=(GPUEXP_BENCH_EXPORTER_ROOT=$PWD/ab_r02) ;;
      idle_cont) envs=(GPUEXP_COUNTERS_KICK=start); extra=(--busy 0) ;;
      idle_off) extra=(--counters 0 --busy 0) ;;
      *) echo "unknown arm $arm"; exit 2 ;;
    esac
    echo "[ab] rep $rep arm $arm $(date +%T)"
    rc=0
    env "${envs[@]}" timeout -k 10 180 python -u bench.py --steps 40 --warmup 5 --identity-phase 0 \
      "${extra[@]}" --out "gpurun_out/ab/$arm.$rep.json" > "gpurun_out/ab/$arm.$rep.out" 2> "gpurun_out/ab/$arm.$rep.err" || rc=$?
    # rc 1 = the run flagged a problem (its --out JSON says which): keep going; anything else
    # (timeout, abort, crash) ends the A/B
    if [ $rc -ne 0 ]; then
      echo "[ab] $arm.$rep rc=$rc: $(grep -h FAILED gpurun_out/ab/$arm.$rep.err | head -3)"
      [ $rc -eq 1 ] || exit $rc
    fi
    python3 - "$arm" "$rep" <<'PY'
import json, sys
r = json.load(open(f"gpurun_out/ab/{sys.argv[1]}.{sys.argv[2]}.json"))
print("[ab]", sys.argv[1], sys.argv[2], "p50", r["value"], "cpu%", r["exporter_cpu_percent"],
      "devices", r["sample_stage_mean_us"].get("devices"), "sampler/tick", r.get("sampler_cpu_us_per_tick"),
      "parts", r.get("device_read_mean_us_per_tick"), "fetch_cpu", r.get("gpu_metrics_fetch_cpu_us_per_fresh_read_gpu0"),
      "reads", r.get("gpu_metrics_reads_gpu0"), flush=True)
PY
  done
done
