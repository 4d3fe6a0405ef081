// lt_kernels.h — the analyze and resolve kernels (bodies in lt_kernels_dev.h) and the launch of
// one (MAXY, RMAX) instance pair. Included by the dispatch translation units only
// (lt_dispatch_unit.hip: every instance the product needs; the profiling units of profiles/: one
// instance with a phase probe).
//
// Replaces, per pixel tile, the per-grid-point loop of MRLandTrendrJob.analysis_reducer
// (/root/reference/mr_land_trendr_job.py:83-126) around utils.analyze + utils.change_labeling.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lt_kernels_dev.h"
#include "lt_launch.h"

namespace lt {

// WAVES: the waves per SIMD the instance is built for (<= 128 VGPRs at 4)
template <int MAXY, int RMAX, class VT, int WAVES, class Probe>
__global__ __launch_bounds__(64, WAVES) void analyze_fast_kernel(const KernelArgs A) {
  (void)A;  // read through args()
  analyze_body<MAXY, RMAX, VT, Probe>();
}

// Built for 4 waves per SIMD like the analyze kernel (<= 128 VGPRs; the compiler's own choice
// was 170, 2 waves): each resolve wave beside the next tile's analyze launch then holds the
// registers of one analyze wave, not two (c2 21.62 vs 21.67 ms per step, profiles/r04_run3).
template <int MAXY, int RMAX, class VT>
__global__ __launch_bounds__(64, 4) void resolve_fast_kernel(const KernelArgs A) {
  (void)A;  // read through args()
  resolve_body<MAXY, RMAX, VT>();
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
  return KernelArgs{l.scene, *l.params, *l.in, *l.out, l.xtab, defer, counters, l.yflags,
                    l.tl_bits, l.tl_eqn};
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
