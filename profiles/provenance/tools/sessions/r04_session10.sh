#!/bin/bash
# Round-4 GPU session 10: HTTP pre-wake slice A/B on another box, 3 interleaved reps of
# 100 scrapes per arm: slices of 150 us (current default) / 300 us / 500 us / pre-wake off.
# (session 9: menu governor, C1 2 us / C2 200 us target residency; p50 80/80 us at 150 us
# slices vs 32/23 at 300 us vs 40/42 off.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s10
B="python -u bench.py --gpus 1 --steps 100 --warmup 10 --identity-phase 0"
steps=("30::{ cat /sys/devices/system/cpu/cpuidle/current_governor_ro 2>/dev/null; for s in /sys/devices/system/cpu/cpu0/cpuidle/state*; do echo \$(cat \$s/name) latency_us=\$(cat \$s/latency) residency_us=\$(cat \$s/residency); done; } > gpurun_out/r04s10/cpuidle.txt 2>&1; cat gpurun_out/r04s10/cpuidle.txt")
for rep in 1 2 3; do
  steps+=("150::GPUEXP_HTTP_PREWAKE_STEP_US=150 $B --out gpurun_out/r04s10/p150.$rep.json")
  steps+=("150::GPUEXP_HTTP_PREWAKE_STEP_US=300 $B --out gpurun_out/r04s10/p300.$rep.json")
  steps+=("150::GPUEXP_HTTP_PREWAKE_STEP_US=500 $B --out gpurun_out/r04s10/p500.$rep.json")
  steps+=("150::GPUEXP_HTTP_PREWAKE=false $B --out gpurun_out/r04s10/off.$rep.json")
done
bash tools/gpu_session.sh "${steps[@]}"
