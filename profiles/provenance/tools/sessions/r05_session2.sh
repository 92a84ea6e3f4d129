#!/bin/bash
# Round-5 GPU session 2: BASELINE config 5 (100 Hz) with the compiled vs the classic exposition,
# interleaved (VERDICT r04 task 2); pre-wake on/off at the driver's command, 5 interleaved pairs
# (task 4); one rocprofv3 kernel-trace of the driver's command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s2
mkdir -p $O
C5="python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0"
D="python -u bench.py --gpus 1 --steps 20 --warmup 5"
steps=()
for i in 1 2 3; do
  steps+=("200::$C5 --out $O/c5_compiled.$i.json")
  steps+=("200::GPUEXP_EXPOSITION=classic $C5 --out $O/c5_classic.$i.json")
done
for i in 1 2 3 4 5; do
  steps+=("150::$D --out $O/driver_prewake_on.$i.json")
  steps+=("150::GPUEXP_HTTP_PREWAKE=0 $D --out $O/driver_prewake_off.$i.json")
done
steps+=("240::cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && rocprofv3 --kernel-trace --stats -d $O/rocprof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --out $O/rocprof_bench.json > $O/rocprof.log 2>&1; tail -5 $O/rocprof.log")
bash tools/gpu_session.sh "${steps[@]}"
