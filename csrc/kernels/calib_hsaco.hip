// Stand-alone code object (gpuexp_calib.hsaco, device-only for gfx950) with the PMC
// calibration workloads under C names, dispatched as raw AQL packets on the aqlprofile
// plugin's own PMC queue by gpuexp_rp_calibrate (aql_pmc.cc).  Agent-mode SQ/TCC counters
// of an unprivileged process count only that queue's dispatches (profiles/r02/pmc_scope.txt),
// so this is where known work can be held against the derived families.
#include "kernels/probe_device.h"

extern "C" __global__ void __launch_bounds__(gpuexp::kProbeBlock) gpuexp_calib_copy(gpuexp::CalibCopyArgs a) {
  gpuexp::stream_copy_body(static_cast<const gpuexp::u32x4*>(a.src), static_cast<gpuexp::u32x4*>(a.dst), a.n,
                           a.blocks);
}

extern "C" __global__ void __launch_bounds__(gpuexp::kProbeBlock) gpuexp_calib_lds(gpuexp::CalibLdsArgs a) {
  gpuexp::lds_probe_body(a.out, a.iters, a.stride);
}

extern "C" __global__ void __launch_bounds__(gpuexp::kProbeBlock) gpuexp_calib_mfma(gpuexp::CalibMfmaCountArgs a) {
  gpuexp::mfma_count_body(a);
}
