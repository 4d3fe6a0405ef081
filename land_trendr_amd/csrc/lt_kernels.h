// lt_kernels.h — the analyze and resolve kernels around the wave-lockstep body of lt_fast.h, and
// the launch of one (MAXY, RMAX) instance pair. Included by the dispatch translation units only
// (lt_dispatch.hip: every instance the product needs; the profiling units of profiles/: one
// instance with a phase probe).
//
// Replaces, per pixel tile, the per-grid-point loop of MRLandTrendrJob.analysis_reducer
// (/root/reference/mr_land_trendr_job.py:83-126) around utils.analyze + utils.change_labeling.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lt_fast.h"
#include "lt_launch.h"

namespace lt {

__device__ inline void defer_append(bool deferred, int64_t p, int lane, int64_t* __restrict__ list,
                                    unsigned long long* __restrict__ count) {
  const uint64_t mask = __ballot(deferred);
  if (mask == 0) return;
  const int leader = __ffsll((long long)mask) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(count, (unsigned long long)__popcll(mask));
  base = __shfl(base, leader);
  if (deferred) list[base + __popcll(mask & ((1ull << lane) - 1))] = p;
}

// Every argument of the analyze / resolve kernels, passed as ONE by-value struct. The kernels read
// its fields through the kernarg segment pointer at their uses (args()), so a field is loaded
// where a stage needs it: a kernel that names its by-value parameters gets every one of them
// loaded into SGPRs at entry (AMDGPU lowers kernel arguments there), and the ~60 SGPRs of tile
// pointers and rule fields then live through the DP as SGPR spills in VGPR lanes (a lane VGPR
// taken from the DP, a v_readlane per use).
struct KernelArgs {
  const DevScene* S;
  lt_params P;
  lt_tile_in in;
  lt_tile_out out;
  const lsq_xf* xtab;
  int64_t* defer;
  unsigned long long* n_defer;  // analyze: [0]/[2] list counts; resolve: its counters
  uint64_t* yflags;
};

__device__ inline const KernelArgs& args() {
  return *(const KernelArgs*)__builtin_amdgcn_kernarg_segment_ptr();
}

// Stage 1 (wave-lockstep body, lt_fast.h): one wave per workgroup, the pixel series in LDS.
// WAVES: the waves per SIMD the instance is built for (<= 128 VGPRs at 4). VT: the LDS type of
// the series — int16 when the tile's index raster is int16 (every value fits; half the LDS of
// binary32, so more waves per CU), binary64 for binary64 values, else binary32 (values it cannot
// hold defer the pixel to the binary64 resolve). Probe: lt_fast.h's phase probe (NoProbe here;
// the profiling units of profiles/ pass theirs).
template <int MAXY, int RMAX, class VT, int WAVES, class Probe>
__global__ __launch_bounds__(64, WAVES) void analyze_fast_kernel(const KernelArgs A) {
  (void)A;  // read through args()
  __shared__ WaveLds<MAXY, VT, false> L;
  const KernelArgs& K = args();
  const int lane = threadIdx.x;
  const int64_t p = (int64_t)blockIdx.x * 64 + lane;
  const int64_t n_pix = K.in.n_pix;
  const bool live = p < n_pix;
  const int d = analyze_fast<MAXY, RMAX, false, VT>(*K.S, K.P, K.in, K.out, K.xtab, K.yflags, p,
                                                    live, lane, L, Probe{});
  // two lists: [0, n_pix) for the binary32 resolve, [n_pix, 2 n_pix) for the binary64 one;
  // counters [0] / [2] count them (wave-aggregated atomics)
  const KernelArgs& K2 = args();
  defer_append(live && d == kDeferExact, p, lane, K2.defer, &K2.n_defer[0]);
  defer_append(live && d == kDeferWide, p, lane, K2.defer + K2.in.n_pix, &K2.n_defer[2]);
}

// Stage 2 (wave-lockstep, lt_fast.h with EXACT): the deferred pixels, binary64 series in LDS,
// exact-OPT DP. A grid of exactly the resident waves takes 64-pixel groups of the list from a
// counter (group cost varies a lot); every wave leaves once the counter has passed the list.
template <int MAXY, int RMAX, class VT>
__global__ __launch_bounds__(64) void resolve_fast_kernel(const KernelArgs A) {
  (void)A;  // read through args()
  __shared__ WaveLds<MAXY, VT, true> L;
  const int lane = threadIdx.x;
  const KernelArgs& K = args();
  unsigned long long* counters = K.n_defer;
  const int64_t n = (int64_t)counters[0];  // written by stage 1, a previous launch
  for (;;) {
    unsigned g = 0;
    if (lane == 0) g = atomicAdd((unsigned*)&counters[1], 1u);
    g = __builtin_amdgcn_readfirstlane(__shfl(g, 0));
    const int64_t base = (int64_t)g * 64;
    if (base >= n) break;
    const int64_t k = base + lane;
    const bool live = k < n;
    const KernelArgs& Kk = args();
    analyze_fast<MAXY, RMAX, true, VT>(*Kk.S, Kk.P, Kk.in, Kk.out, Kk.xtab, Kk.yflags,
                                       live ? Kk.defer[k] : 0, live, lane, L);
  }
}

// waves of resolve_fast_kernel<MAXY, RMAX, VT> the device holds at once
template <int MAXY, int RMAX, class VT>
inline unsigned resolve_grid(int device) {
  static int cached_dev = -1;
  static unsigned cached = 0;
  if (cached_dev != device) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, resolve_fast_kernel<MAXY, RMAX, VT>,
                                                     64, 0) != hipSuccess || per_cu < 1)
      per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
        cus < 1)
      cus = 256;
    cached = (unsigned)(per_cu * cus);
    cached_dev = device;
  }
  return cached;
}

// the tile's series type: int16 for an int16 index raster; binary64 for binary64 values (obs_val
// or an f64 index raster) with up to 4 rules — the lazy DP on a binary64 LDS series, where
// otherwise every value binary32 cannot hold would send its pixel to the exact-OPT resolve stage
// (46 vs 1842 Mpx/s, profiles/float_index.py); else binary32
enum SeriesKind { kSeriesI16, kSeriesF64, kSeriesF32 };
// (the fused load stage: its values are those of an index raster of type lin.out_type)
inline SeriesKind series_kind(const TileLaunch& l) {
  const bool raster = l.in->obs_index || l.in->obs_bands;
  const int t = l.in->obs_bands ? l.in->lin.out_type : l.in->index_type;
  if (raster && t == LT_T_I16) return kSeriesI16;
  if ((!raster || t == LT_T_F64) && l.params->n_rules <= 4) return kSeriesF64;
  return kSeriesF32;
}

inline dim3 tile_grid(const TileLaunch& l) { return dim3((unsigned)((l.in->n_pix + 63) / 64)); }

inline KernelArgs kernel_args(const TileLaunch& l, int64_t* defer, unsigned long long* counters) {
  return KernelArgs{l.scene, *l.params, *l.in, *l.out, l.xtab, defer, counters, l.yflags};
}

template <int MAXY, int RMAX, int WAVES, class Probe>
hipError_t launch_analyze_instance(const TileLaunch& l) {
  const dim3 grid = tile_grid(l), block(64);
  const SeriesKind k = series_kind(l);
  const KernelArgs a = kernel_args(l, l.defer, l.counters);
  if (k == kSeriesI16) {
    hipLaunchKernelGGL((analyze_fast_kernel<MAXY, RMAX, int16_t, WAVES, Probe>), grid, block, 0,
                       l.stream, a);
  } else if (k == kSeriesF64) {
    if constexpr (RMAX <= 4)  // the binary64 analyze instance exists for up to 4 rules
      hipLaunchKernelGGL((analyze_fast_kernel<MAXY, RMAX, double, WAVES, Probe>), grid, block, 0,
                         l.stream, a);
  } else {
    hipLaunchKernelGGL((analyze_fast_kernel<MAXY, RMAX, float, WAVES, Probe>), grid, block, 0,
                       l.stream, a);
  }
  return hipGetLastError();
}

template <int MAXY, int RMAX, class VT>
void launch_resolve1(const TileLaunch& l, int64_t* list, unsigned long long* counters) {
  const unsigned g = resolve_grid<MAXY, RMAX, VT>(l.device);
  const int64_t nwave = (l.in->n_pix + 63) / 64;
  const dim3 grid((unsigned)(nwave < (int64_t)g ? nwave : (int64_t)g)), block(64);
  hipLaunchKernelGGL((resolve_fast_kernel<MAXY, RMAX, VT>), grid, block, 0, l.stream,
                     kernel_args(l, list, counters));
}

// both deferred lists: the first in the tile's series type, the second (values binary32 cannot
// hold) in binary64. An int16 series is exact in binary32, so its second list is always empty and
// is not launched: the launch's resident-size grid of waves that find nothing to do still took
// CU slots beside the next tile's analyze waves (3.9 ms of trace time per tile on c2,
// profiles/r03_c2_kernel_stats_head.csv)
template <int MAXY, int RMAX>
hipError_t launch_resolve_instance(const TileLaunch& l) {
  const SeriesKind k = series_kind(l);
  if (k == kSeriesI16) launch_resolve1<MAXY, RMAX, int16_t>(l, l.defer, l.counters);
  else if (k == kSeriesF64) launch_resolve1<MAXY, RMAX, double>(l, l.defer, l.counters);
  else launch_resolve1<MAXY, RMAX, float>(l, l.defer, l.counters);
  if (k != kSeriesI16)
    launch_resolve1<MAXY, RMAX, double>(l, l.defer + l.in->n_pix, l.counters + 2);
  return hipGetLastError();
}

}  // namespace lt
