#!/bin/bash
# Round-4 GPU session 9: the box's CPU idle states (what the HTTP pre-wake slices must stay
# under), then the pre-wake A/B at 100 scrapes per run: slices of 150 us (default) / 300 us /
# pre-wake off, interleaved x2.  First a driver-form run of the tree (bench now signals the
# exporter after writing its pod map instead of a 0.5 s control-plane poll).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s9
B="python -u bench.py --gpus 1 --steps 100 --warmup 10 --identity-phase 0"
bash tools/gpu_session.sh \
  "30::{ cat /sys/devices/system/cpu/cpuidle/current_governor_ro 2>/dev/null || cat /sys/devices/system/cpu/cpuidle/current_governor; for s in /sys/devices/system/cpu/cpu0/cpuidle/state*; do echo \$(cat \$s/name) latency_us=\$(cat \$s/latency) residency_us=\$(cat \$s/residency) disabled=\$(cat \$s/disable); done; nproc; } > gpurun_out/r04s9/cpuidle.txt 2>&1; cat gpurun_out/r04s9/cpuidle.txt" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s9/bench_driver_form.json" \
  "150::$B --out gpurun_out/r04s9/p150.1.json" \
  "150::GPUEXP_HTTP_PREWAKE_STEP_US=300 $B --out gpurun_out/r04s9/p300.1.json" \
  "150::GPUEXP_HTTP_PREWAKE=false $B --out gpurun_out/r04s9/off.1.json" \
  "150::$B --out gpurun_out/r04s9/p150.2.json" \
  "150::GPUEXP_HTTP_PREWAKE_STEP_US=300 $B --out gpurun_out/r04s9/p300.2.json" \
  "150::GPUEXP_HTTP_PREWAKE=false $B --out gpurun_out/r04s9/off.2.json"
