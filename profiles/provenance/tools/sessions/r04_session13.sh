#!/bin/bash
# Round-4 GPU session 13: the occupancy limiters against VGPR- and SGPR-limited kernels too,
# then BASELINE configs 1 (mock backend), 2 (1 Hz) and 5 (100 Hz scrape + sample) on the final
# tree, plus two more driver-form runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04s13
bash tools/gpu_session.sh \
  "200::python -u tools/probe_spi_scope.py --seconds 2.0 --no-self --exported --kinds lds,waves,vgpr,sgpr > gpurun_out/r04s13/spi_limiters.log 2>&1; grep -E '^(idle|lds_|waves_|vgpr_|sgpr_)' gpurun_out/r04s13/spi_limiters.log | cut -c1-330" \
  "200::python -u bench.py --sample-hz 100 --scrape-hz 100 --steps 1000 --warmup 100 --identity-phase 0 --out gpurun_out/r04s13/bench_config5_100hz.json" \
  "200::python -u bench.py --sample-hz 1 --scrape-hz 1 --steps 30 --warmup 3 --identity-phase 0 --out gpurun_out/r04s13/bench_config2_1hz.json" \
  "200::python -u bench.py --backend mock --steps 100 --warmup 10 --out gpurun_out/r04s13/bench_config1_mock.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s13/bench_driver_form_4.json" \
  "150::python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04s13/bench_driver_form_5.json"
