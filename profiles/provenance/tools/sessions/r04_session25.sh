#!/bin/bash
# Round-4 GPU session 25: the driver's bench command 10 times back to back on one box (the
# distribution a single end-of-round run draws from).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s25
steps=()
for i in $(seq 1 10); do
  steps+=("150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s25/bench_driver_form_$i.json")
done
bash tools/gpu_session.sh "${steps[@]}"
