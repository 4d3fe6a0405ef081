// stamp_probe.h — PROFILING BUILD ONLY (profiles/stamps.sh force-includes it into the profiling
// dispatch unit with LT_PROBE=StampProbe). Per phase of analyze_fast (lt_fast.h probe.mark), the
// shader cycles each wave spends there (s_memtime deltas), summed over waves with one atomic per
// wave and phase, plus the wave count. Results unchanged: the probe only reads the clock.
#pragma once
#include <hip/hip_runtime.h>

__device__ unsigned long long lt_stamp_cycles[8];

struct StampProbe {
  static constexpr int kStopAfter = -1;
  mutable unsigned long long t;
  __device__ StampProbe() : t(__builtin_amdgcn_s_memtime()) {}
  __device__ void mark(int k) const {
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
      atomicAdd(&lt_stamp_cycles[k], now - t);
      if (k == 4) atomicAdd(&lt_stamp_cycles[7], 1ull);
    }
    t = now;
  }
};

extern "C" int lt_diag_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lt_stamp_cycles), sizeof(unsigned long long) * 8) !=
      hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(lt_stamp_cycles), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
