// Stand-alone code object (gpuexp_sentinel.hsaco, built device-only for gfx950) with the
// sentinel's entry points under C names and by-value argument structs, for hosts that
// dispatch raw AQL packets instead of going through HIP (aql_pmc.cc: the sentinel shares
// the counters' HSA queue).  Same device code as the HIP plugin (sentinel_device.h).
#include "gpuexp/sentinel_device.h"

extern "C" __global__ void __launch_bounds__(64) gpuexp_sentinel(gpuexp::SentinelArgs a) {
  gpuexp::sentinel_body(a.ring, a.slot, a.seq, a.spin, a.chase, a.hops);
}

extern "C" __global__ void __launch_bounds__(64) gpuexp_sentinel_init_chase(gpuexp::SentinelInitArgs a) {
  gpuexp::sentinel_init_chase_body(a.chase, a.hops);
}
