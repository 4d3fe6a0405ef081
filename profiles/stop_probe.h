// stop_probe.h — PROFILING BUILDS ONLY (profiles/phases.sh force-includes it into the profiling
// dispatch unit, LT_PROBE=StopProbe<K>): the analyze kernel cut after phase K (lt_fast.h probe), so
// PMC counts of builds K = 0..3 and of the product give each phase's instructions by difference.
#pragma once
template <int K>
struct StopProbe {
  static constexpr int kStopAfter = K;
  __device__ void mark(int) const {}
};
