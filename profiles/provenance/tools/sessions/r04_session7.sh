#!/bin/bash
# Round-4 GPU session 7: (1) the PMC GPU tests with inline rounds plus the follow-up of reads
# that outlive the sync wait; (2) the driver's bench command per arm, interleaved:
#   A  thread-run PMC rounds, HTTP worker unpinned   (the session-5 tree's behaviour)
#   B  inline PMC rounds
#   C  inline PMC rounds + HTTP worker following the scraper's receive CPU
# (3) the unit of KFD's per-process sdma_<id> file (child found by its KFD host PID).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s7
A="GPUEXP_PMC_INLINE=0 GPUEXP_HTTP_FOLLOW_RX_CPU=0"
B="GPUEXP_PMC_INLINE=1 GPUEXP_HTTP_FOLLOW_RX_CPU=0"
C="GPUEXP_PMC_INLINE=1 GPUEXP_HTTP_FOLLOW_RX_CPU=1"
BENCH="python -u bench.py --gpus 1 --steps 20 --warmup 5"
bash tools/gpu_session.sh \
  "300::GPUEXP_PMC_INLINE=1 python -u -m pytest tests/test_gpu.py -x -v --timeout 240 --timeout-method thread -k 'counters or calibration or limiters or exporter_tick or devices_stage' > gpurun_out/r04s7/pytest_pmc.log 2>&1; tail -4 gpurun_out/r04s7/pytest_pmc.log" \
  "150::env $A $BENCH --out gpurun_out/r04s7/A.1.json" \
  "150::env $B $BENCH --out gpurun_out/r04s7/B.1.json" \
  "150::env $C $BENCH --out gpurun_out/r04s7/C.1.json" \
  "150::env $A $BENCH --out gpurun_out/r04s7/A.2.json" \
  "150::env $B $BENCH --out gpurun_out/r04s7/B.2.json" \
  "150::env $C $BENCH --out gpurun_out/r04s7/C.2.json" \
  "150::env $C python -u bench.py --gpus 1 --steps 100 --warmup 10 --out gpurun_out/r04s7/C.100.json" \
  "150::env $A python -u bench.py --gpus 1 --steps 100 --warmup 10 --out gpurun_out/r04s7/A.100.json" \
  "90::python -u tools/probe_sdma_units.py --seconds 1.5 > gpurun_out/r04s7/sdma_units.log 2>&1; grep -v RESULT gpurun_out/r04s7/sdma_units.log | cut -c1-300"
