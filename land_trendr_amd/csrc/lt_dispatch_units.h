// lt_dispatch_units.h — the per-(MAXY, RMAX) launch functions of the product's analyze / resolve
// instances. Each is defined in its own translation unit (lt_dispatch_unit.hip compiled with
// -DLT_UNIT_MAXY=<MAXY> -DLT_UNIT_RMAX=<RMAX>); lt_dispatch.hip picks one per tile.
#pragma once
#include "lt_launch.h"

namespace lt {

template <int MAXY, int RMAX>
hipError_t analyze_unit(const TileLaunch& l);
template <int MAXY, int RMAX>
hipError_t resolve_unit(const TileLaunch& l);

#define LT_DECLARE_UNIT(MY, RM)                                  \
  template <> hipError_t analyze_unit<MY, RM>(const TileLaunch&); \
  template <> hipError_t resolve_unit<MY, RM>(const TileLaunch&);
LT_DECLARE_UNIT(32, 1)
LT_DECLARE_UNIT(32, 4)
LT_DECLARE_UNIT(32, 16)
LT_DECLARE_UNIT(48, 1)
LT_DECLARE_UNIT(48, 4)
LT_DECLARE_UNIT(48, 16)
LT_DECLARE_UNIT(64, 1)
LT_DECLARE_UNIT(64, 4)
LT_DECLARE_UNIT(64, 16)
#undef LT_DECLARE_UNIT

}  // namespace lt
