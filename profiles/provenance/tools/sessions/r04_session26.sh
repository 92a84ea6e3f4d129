#!/bin/bash
# Round-4 GPU session 26: the driver's bench command 10 times on another box, then BASELINE
# config 5 (100 Hz) twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s26
steps=()
for i in $(seq 1 10); do
  steps+=("150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s26/bench_driver_form_$i.json")
done
for i in 1 2; do
  steps+=("200::python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0 --out gpurun_out/r04s26/bench_config5_$i.json")
done
bash tools/gpu_session.sh "${steps[@]}"
