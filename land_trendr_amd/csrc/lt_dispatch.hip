// lt_dispatch.hip — the product's analyze / resolve instances (lt_kernels.h), chosen per tile by
// the scene's year count (MAXY: the LDS series and DP arrays are sized for it) and the rule count
// (RMAX: per-rule state in registers; up to LT_CERT_RULES rules take the certified labels path).
#include "lt_kernels.h"

namespace lt {

namespace {
// waves per SIMD each instance is built for: 4 (<= 128 VGPRs) where the body fits without
// spilling (5 for the c2 instance was measured slower: 1365 vs 2079 Mpx/s, spills)
constexpr int kWaves = 4;

template <int MAXY>
hipError_t analyze_for(const TileLaunch& l) {
  const int r = l.params->n_rules;
  if (r <= 1) return launch_analyze_instance<MAXY, 1, kWaves, NoProbe>(l);
  if (r <= 4) return launch_analyze_instance<MAXY, 4, kWaves, NoProbe>(l);
  return launch_analyze_instance<MAXY, 16, kWaves, NoProbe>(l);
}

template <int MAXY>
hipError_t resolve_for(const TileLaunch& l) {
  const int r = l.params->n_rules;
  if (r <= 1) return launch_resolve_instance<MAXY, 1>(l);
  if (r <= 4) return launch_resolve_instance<MAXY, 4>(l);
  return launch_resolve_instance<MAXY, 16>(l);
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
