// lt_dispatch_probe.hip — PROFILING / A-B BUILDS ONLY. Stands in for the product's dispatch unit
// (land_trendr_amd/csrc/lt_dispatch.hip) in a library linked from lt_abi.hip and this file: one
// analyze / resolve instance (LT_PROBE_MAXY years, LT_PROBE_RMAX rules, default one) with the phase probe LT_PROBE
// (profiles/stamp_probe.h, stop_probe.h, force-included by the build scripts).
#include "../land_trendr_amd/csrc/lt_kernels.h"

#ifndef LT_PROBE
#define LT_PROBE lt::NoProbe
#endif
#ifndef LT_PROBE_MAXY
#define LT_PROBE_MAXY 32
#endif
#ifndef LT_PROBE_RMAX
#define LT_PROBE_RMAX 1
#endif
#ifndef LT_PROBE_WAVES
#define LT_PROBE_WAVES 4
#endif

namespace lt {
hipError_t launch_analyze(const TileLaunch& l) {
  return launch_analyze_instance<LT_PROBE_MAXY, LT_PROBE_RMAX, LT_PROBE_WAVES, LT_PROBE>(l);
}
hipError_t launch_resolve(const TileLaunch& l) { return launch_resolve_instance<LT_PROBE_MAXY, LT_PROBE_RMAX>(l); }
}  // namespace lt
