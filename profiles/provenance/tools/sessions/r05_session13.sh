#!/bin/bash
# Round-5 GPU session 13: one rocprofv3 kernel trace of the driver's command on the final tree
# (the sentinel's per-dispatch time on the PMC queue, the GEMM pod's kernels).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s13
mkdir -p $O
bash tools/gpu_session.sh \
  "240::cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && rocprofv3 --kernel-trace --stats -d $O/rocprof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --out $O/rocprof_bench.json > $O/rocprof.log 2>&1; tail -5 $O/rocprof.log"
