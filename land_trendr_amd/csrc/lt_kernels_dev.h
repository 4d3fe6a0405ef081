// lt_kernels_dev.h — device side of the analyze / resolve kernels: their one by-value argument
// struct and their bodies around the wave-lockstep analysis of lt_fast.h. Included by lt_kernels.h
// (the product's __global__ instances and their launches) and by the JIT kernels of lt_jit.h
// (hiprtc, an index_eqn program inlined into the winner pick), which therefore share the
// argument layout and the code.
//
// Replaces, per pixel tile, the per-grid-point loop of MRLandTrendrJob.analysis_reducer
// (/root/reference/mr_land_trendr_job.py:83-126) around utils.analyze + utils.change_labeling.
#pragma once
#include "lt_fast.h"

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

// The pixel group of workgroup b (64 pixels each). LT_XCD_REMAP = 1: blocks are dealt round-robin
// over the 8 XCDs (MI355X_MICROARCH.md § Workgroup dispatch, observed placement, speed only), so the
// blocks sharing an XCD (equal b % 8) take one contiguous pixel range, in order: consecutive
// groups' row pieces of a per-year plane then leave the same L2 close in time. 0: group b.
#ifndef LT_XCD_REMAP
#define LT_XCD_REMAP 0
#endif
__device__ inline int64_t xcd_block(unsigned b, unsigned G) {
  if (!LT_XCD_REMAP) return (int64_t)b;
  const unsigned x = b & 7u, i = b >> 3, q = G >> 3, r = G & 7u;  // bijective for any G
  return (int64_t)x * q + (x < r ? x : r) + i;
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
  uint64_t* tl_bits;  // the compact trendline (lt_fast.h tl_split), or null
  double* tl_eqn;
};

__device__ inline const KernelArgs& args() {
  return *(const KernelArgs*)__builtin_amdgcn_kernarg_segment_ptr();
}

// Stage 1 (wave-lockstep body, lt_fast.h): one wave per workgroup, the pixel series in LDS.
// VT: the LDS type of the series — int16 when the tile's index raster is int16 (every value
// fits; half the LDS of
// binary32, so more waves per CU), binary64 for binary64 values, else binary32 (values it cannot
// hold defer the pixel to the binary64 resolve). Probe: lt_fast.h's phase probe (NoProbe here;
// the profiling units of profiles/ pass theirs).
// LT_WPB: waves per workgroup (the JIT kernels, lt_jit.h analyze_wpb; the precompiled instances 1):
// each wave has its own LDS slice and 64 pixels; a workgroup takes 64 * LT_WPB consecutive pixels
#ifndef LT_WPB
#define LT_WPB 1
#endif
template <int MAXY, int RMAX, class VT, class Probe>
__device__ inline void analyze_body() {
  __shared__ WaveLds<MAXY, VT, false> Ls[LT_WPB];
  WaveLds<MAXY, VT, false>& L = Ls[LT_WPB > 1 ? threadIdx.x >> 6 : 0];
  const KernelArgs& K = args();
  const int lane = LT_WPB > 1 ? threadIdx.x & 63 : threadIdx.x;
#ifdef LT_DEBUG_LDS_PAD
  // debugging (LT_JIT_DEFINES=LT_DEBUG_LDS_PAD=bytes): extra LDS per workgroup, to run the
  // analyze stage at a lower occupancy (fewer co-resident waves per CU) with the same code
  __shared__ uint32_t lds_pad[LT_DEBUG_LDS_PAD / 4];
  lds_pad[lane] = (uint32_t)lane;
  asm volatile("" ::"v"(lds_pad[lane]));
#endif
  const int64_t p = xcd_block(blockIdx.x, gridDim.x) * (64 * LT_WPB) + threadIdx.x;
  const int64_t n_pix = K.in.n_pix;
#if defined(LT_SPEC_FULL) && LT_SPEC_FULL
  // the tile is whole waves (lt_jit.h Spec::full): every lane has a pixel
  const bool live = true;
  (void)n_pix;
#else
  const bool live = p < n_pix;
#endif
  const int d = analyze_fast<MAXY, RMAX, false, VT>(*K.S, K.P, K.in, K.out, K.xtab, K.yflags,
                                                    K.tl_bits, K.tl_eqn, p, live, lane, L,
                                                    Probe{});
  // two lists: [0, n_pix) for the binary32 resolve, [n_pix, 2 n_pix) for the binary64 one;
  // counters [0] / [2] count them (wave-aggregated atomics)
  const KernelArgs& K2 = args();
  defer_append(live && d == kDeferExact, p, lane, K2.defer, &K2.n_defer[0]);
  defer_append(live && d == kDeferWide, p, lane, K2.defer + K2.in.n_pix, &K2.n_defer[2]);
}

// Stage 2 (wave-lockstep, lt_fast.h with EXACT): the deferred pixels (list n_defer[0] of
// `defer`). A grid of exactly the resident waves takes groups of LT_RESOLVE_GROUP pixels of the
// list from a counter (group cost varies a lot); every wave leaves once the counter has passed the
// list. A group smaller than the wave leaves lanes idle but splits the list finer: the stage is a
// few thousand latency-bound waves, so its time is that of its slowest wave.
// For an int16 series the list of values binary32 cannot hold ([n_pix, 2 n_pix)) is empty.
#ifndef LT_RESOLVE_GROUP
#define LT_RESOLVE_GROUP 64
#endif
template <int MAXY, int RMAX, class VT>
__device__ inline void resolve_body() {
  __shared__ WaveLds<MAXY, VT, true> L;
  constexpr int G = LT_RESOLVE_GROUP;
  static_assert(G >= 1 && G <= 64, "a group is at most one wave");
  const int lane = threadIdx.x;
  const KernelArgs& K = args();
  unsigned long long* counters = K.n_defer;
  const int64_t n = (int64_t)counters[0];  // written by stage 1, a previous launch
  for (;;) {
    unsigned g = 0;
    if (lane == 0) g = atomicAdd((unsigned*)&counters[1], 1u);
    g = __builtin_amdgcn_readfirstlane(__shfl(g, 0));
    const int64_t base = (int64_t)g * G;
    if (base >= n) break;
    const int64_t k = base + lane;
    const bool live = lane < G && k < n;
    const KernelArgs& Kk = args();
    analyze_fast<MAXY, RMAX, true, VT>(*Kk.S, Kk.P, Kk.in, Kk.out, Kk.xtab, Kk.yflags,
                                       Kk.tl_bits, Kk.tl_eqn, live ? Kk.defer[k] : 0, live, lane,
                                       L);
  }
}

}  // namespace lt
