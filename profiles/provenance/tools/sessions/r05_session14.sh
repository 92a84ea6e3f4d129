#!/bin/bash
# Round-5 GPU session 14: does the ROCr utility queue (and its 173 MiB context save area) still
# appear when the exporter's queue asks for no private / group segment?  tools/probe_queue_mem.cc,
# one queue, UINT32_MAX (as aql_pmc.cc today) vs 0; plus the same after a code-object load.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s14
mkdir -p $O
g++ -O2 -std=c++17 -I/opt/rocm/include -o $O/probe_queue_mem tools/probe_queue_mem.cc -L/opt/rocm/lib -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib || exit 1
bash tools/gpu_session.sh \
  "60::$O/probe_queue_mem 1 > $O/seg_max.log 2>&1; cat $O/seg_max.log" \
  "60::GPUEXP_PROBE_SEG=0 $O/probe_queue_mem 1 > $O/seg_zero.log 2>&1; cat $O/seg_zero.log" \
  "60::GPUEXP_PROBE_SEG=0 $O/probe_queue_mem 1 kubernetes_gpu_exporter_amd/gpuexp_sentinel.hsaco > $O/seg_zero_co.log 2>&1; cat $O/seg_zero_co.log"
