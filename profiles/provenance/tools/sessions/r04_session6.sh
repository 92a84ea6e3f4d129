#!/bin/bash
# Round-4 GPU session 6: PMC read rounds run by the sampler (inline, no counting-thread
# wake-ups) vs by the counting thread; then the unit of KFD's per-process sdma_<id> file.  Counter GPU tests (incl. the starvation / rescue
# case) with inline rounds first, then the driver's bench command interleaved per arm.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s6
bash tools/gpu_session.sh \
  "300::GPUEXP_PMC_INLINE=1 python -u -m pytest tests/test_gpu.py -x -v --timeout 240 --timeout-method thread -k 'counters or calibration or limiters or exporter_tick or devices_stage' > gpurun_out/r04s6/pytest_pmc.log 2>&1; tail -4 gpurun_out/r04s6/pytest_pmc.log" \
  "150::GPUEXP_PMC_INLINE=1 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s6/inline.1.json" \
  "150::GPUEXP_PMC_INLINE=0 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s6/thread.1.json" \
  "150::GPUEXP_PMC_INLINE=1 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s6/inline.2.json" \
  "150::GPUEXP_PMC_INLINE=0 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s6/thread.2.json" \
  "150::GPUEXP_PMC_INLINE=1 python -u bench.py --gpus 1 --steps 100 --warmup 10 --out gpurun_out/r04s6/inline.100.json" \
  "150::GPUEXP_PMC_INLINE=0 python -u bench.py --gpus 1 --steps 100 --warmup 10 --out gpurun_out/r04s6/thread.100.json" \
  "90::python -u tools/probe_sdma_units.py --seconds 1.5 > gpurun_out/r04s6/sdma_units.log 2>&1; grep -v RESULT gpurun_out/r04s6/sdma_units.log | cut -c1-300"
