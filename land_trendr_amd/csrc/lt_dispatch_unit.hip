// lt_dispatch_unit.hip — one (MAXY, RMAX) pair of the product's analyze / resolve instances
// (lt_dispatch_units.h), compiled once per pair with -DLT_UNIT_MAXY=<MAXY> -DLT_UNIT_RMAX=<RMAX>.
#include "lt_dispatch_units.h"
#include "lt_kernels.h"

#if !defined(LT_UNIT_MAXY) || !defined(LT_UNIT_RMAX)
#error "build with -DLT_UNIT_MAXY=<32|48|64> -DLT_UNIT_RMAX=<1|4|16>"
#endif

namespace lt {

// waves per SIMD each instance is built for: 4 (<= 128 VGPRs) where the body fits without
// spilling (5 for the c2 instance was measured slower: 1365 vs 2079 Mpx/s, spills)
constexpr int kWaves = 4;

template <>
hipError_t analyze_unit<LT_UNIT_MAXY, LT_UNIT_RMAX>(const TileLaunch& l) {
  return launch_analyze_instance<LT_UNIT_MAXY, LT_UNIT_RMAX, kWaves, NoProbe>(l);
}

template <>
hipError_t resolve_unit<LT_UNIT_MAXY, LT_UNIT_RMAX>(const TileLaunch& l) {
  return launch_resolve_instance<LT_UNIT_MAXY, LT_UNIT_RMAX>(l);
}

}  // namespace lt
