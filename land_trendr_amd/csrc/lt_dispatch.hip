// lt_dispatch.hip — the product's analyze / resolve instances (lt_kernels.h), chosen per tile by
// the scene's year count (MAXY: the LDS series and DP arrays are sized for it) and the rule count
// (RMAX: per-rule state in registers; up to LT_CERT_RULES rules take the certified labels path).
// Each (MAXY, RMAX) pair is compiled in a translation unit of its own (lt_dispatch_unit.hip, built
// once per pair with -DLT_UNIT_MAXY / -DLT_UNIT_RMAX), so the nine long compiles run side by side.
#include "lt_dispatch_units.h"

namespace lt {

namespace {
template <int MAXY>
hipError_t analyze_for(const TileLaunch& l) {
  const int r = l.params->n_rules;
  if (r <= 1) return analyze_unit<MAXY, 1>(l);
  if (r <= 4) return analyze_unit<MAXY, 4>(l);
  return analyze_unit<MAXY, 16>(l);
}

template <int MAXY>
hipError_t resolve_for(const TileLaunch& l) {
  const int r = l.params->n_rules;
  if (r <= 1) return resolve_unit<MAXY, 1>(l);
  if (r <= 4) return resolve_unit<MAXY, 4>(l);
  return resolve_unit<MAXY, 16>(l);
}
}  // namespace

hipError_t launch_analyze(const TileLaunch& l) {
  if (l.n_years <= 32) return analyze_for<32>(l);
  if (l.n_years <= 48) return analyze_for<48>(l);
  return analyze_for<64>(l);
}

hipError_t launch_resolve(const TileLaunch& l) {
  if (l.n_years <= 32) return resolve_for<32>(l);
  if (l.n_years <= 48) return resolve_for<48>(l);
  return resolve_for<64>(l);
}

}  // namespace lt
