// lt_fast.h — the analyze stage as a wave-lockstep kernel body (one pixel per lane, one wave per
// workgroup). Same results as analyze_pixel<.., true> in lt_pixel.h, organised for CDNA4:
//
//   * per-lane series live in LDS as [index][lane] planes: lane l of element k is at
//     base + (k*64 + l) * sizeof(T), so lanes reading one index k touch consecutive words;
//     lanes at different indices (a per-lane k) can still meet in a bank (PMC: 0.77 conflict
//     cycles per LDS instruction on c2, 0.96 on c3 — small next to ~520 LDS instructions a wave);
//   * loops run over a wave-uniform counter (series position, DP column, vertex number, rule)
//     with per-lane predicates, so the expensive calls (LAPACK-emulated vertex fits) are issued
//     once per vertex NUMBER for the whole wave instead of once per series position per lane;
//   * the DP keeps OPT in registers (static indices from the unrolled inner loop) and decides a
//     column without LAPACK emulation whenever the closed-form prices separate (dp_lazy's rule);
//   * scratch: the analyze stage's OPT values of the DP (OPTa, read at wave-uniform indices
//     below the four-column register window) and a few spills live in per-lane private memory.
#pragma once
#ifndef __HIPCC_RTC__  // hiprtc (the JIT kernels, lt_jit.h) brings its own
#include <type_traits>
#endif

#include "lt_pixel.h"

// winner-pick batch: year slots whose value loads are issued together
#ifndef LT_WB
#define LT_WB 8
#endif
// the exact DP keeps OPT in private memory up to this many years, in registers above
#ifndef LT_RESOLVE_PRIV_MAXY
#define LT_RESOLVE_PRIV_MAXY 48
#endif
// the resolve stage's DP: 1 = the exact-OPT DP over every column (the default), 0 = the lazy DP
// with every ambiguous column decided exactly where it arises (c2 resolve 0.63 vs 0.44 ms per
// launch, 2528 vs 2584 Mpx/s, profiles/r04_run13: the stage is latency-bound, not LAPACK-bound)
#ifndef LT_RESOLVE_FULL
#define LT_RESOLVE_FULL 1
#endif
// timing-only attribution builds (wrong outputs; A/B runs through LT_JIT_DEFINES):
// LT_AB_NO_YEAR_STORES = 1 drops the year-major loop's per-year plane stores, 2 also the winner
// pick's val_raw / winner rows; LT_AB_NO_FITS = 1 drops the year-major loop's emulated fits
#ifndef LT_AB_NO_YEAR_STORES
#define LT_AB_NO_YEAR_STORES 0
#endif
#ifndef LT_AB_NO_FITS
#define LT_AB_NO_FITS 0
#endif
// LT_AB_YEAR_SINK = 1: the year-major loop's plane stores all go to the pixel's year-0 row (the
// same instructions and bytes leave the CUs, ~1/Y of them reach HBM), nontemporal; 2: the same
// with ordinary stores (the rows then stay in L2)
#ifndef LT_AB_YEAR_SINK
#define LT_AB_YEAR_SINK 0
#endif
// the year-major loop's binary64 plane stores: 1 nontemporal (the default), 0 plain
#ifndef LT_YEAR_NT
#define LT_YEAR_NT 1
#endif
// cache policy of the per-year binary64 row stores (year-major planes and val_raw): 0 the
// compiler's nontemporal store (nt: the line stays in the XCD's L2), 1 sc1 (write-through, the
// line dropped from L2: MI355X_MICROARCH.md, store flavours), 2 sc0 sc1, 3 nt sc1
#ifndef LT_YEAR_STORE_MODE
#define LT_YEAR_STORE_MODE 0
#endif

namespace lt {
__device__ inline void year_row_store(double v, double* a) {
#if LT_YEAR_STORE_MODE == 1
  asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(a), "v"(v) : "memory");
#elif LT_YEAR_STORE_MODE == 2
  asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(a), "v"(v) : "memory");
#elif LT_YEAR_STORE_MODE == 3
  asm volatile("global_store_dwordx2 %0, %1, off sc1 nt" ::"v"(a), "v"(v) : "memory");
#else
  __builtin_nontemporal_store(v, a);
#endif
}
}  // namespace lt
// labels-only launches of up to this many rules take the certified path (closed-form fits, the
// emulated ones only around the rules' candidates); more rules keep one emulated fit per vertex
#ifndef LT_CERT_RULES
#define LT_CERT_RULES 4
#endif
// labels-only certified path, pass B: fit only the eqns whose side pass A left undecided, in
// lockstep slots, or all three eqns of every candidate: a stage mask (bit 0 the analyze stage,
// bit 1 the resolve stage: 3 slots in both, 0 in neither)
#ifndef LT_PASSB_SLOTS
#define LT_PASSB_SLOTS 3
#endif

// Launch-uniform values a JIT kernel may be compiled for (lt_jit.h defines LT_SPEC_* for the
// configuration it specialises; the precompiled kernels read them from the launch at run time):
// the rules (LT_SPEC_NRULES rules lt_spec_rules[], pre_threshold mode), the line cost, the year
// count, whether a cloud mask is given, whether any per-year plane is written
#ifdef LT_SPEC_NRULES
#define LT_NRULES LT_SPEC_NRULES
#define LT_RULE(r) lt_spec_rules[r]
#define LT_PRE_MODE LT_SPEC_PRE_MODE
#else
#define LT_NRULES P.n_rules
#define LT_RULE(r) P.rules[r]
#define LT_PRE_MODE P.pre_threshold_mode
#endif
#ifdef LT_SPEC_LINE_COST
#define LT_LINE_COST LT_SPEC_LINE_COST
#else
#define LT_LINE_COST P.line_cost
#endif

namespace lt {

// m * Sxx - Sx^2 of a segment's x sums (m <= 64 points, x <= 255: both products below 2^32, the
// factors below 2^24) with two full-rate 24-bit multiplies instead of two v_mul_lo_u32 (the
// analyze stage's lazy DP; in the resolve stage's exact DP as well it slowed c5's resolve,
// profiles/r04_run27)
__device__ inline int dmul24(int m, int sxx, int sx) {
  return (int)(__umul24((unsigned)m, (unsigned)sxx) - __umul24((unsigned)sx, (unsigned)sx));
}

// max over the 64 lanes of a wave (every lane must call it). readfirstlane makes the result an
// SGPR value, so loops bounded by it are wave-uniform to the compiler: scalar branches instead
// of exec-mask juggling for every test on the loop counter.
__device__ inline int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int u = __shfl_xor(v, o);
    v = u > v ? u : v;
  }
  return __builtin_amdgcn_readfirstlane(v);
}

// Least squares of one segment per active lane, in lockstep: the x half (lsq_factor) comes from
// the device x-set table when the lane's x values are there and is computed only for the lanes
// that miss (a branch the wave takes only if some lane misses); then the y half for every lane.
template <class GX, class GY>
__device__ inline int lsq_lockstep(bool act, int m, GX X, GY Y, const lsq_xf* __restrict__ xtab,
                                   bool need_solution, bool need_ssr, double& slope, double& icpt,
                                   double& ssr) {
  const int key = act ? xset_key(m, X) : 0;
  const bool miss = act && key < 0;
  lsq_xf f;
  if (act && !miss) f = xtab[key];
  if (__ballot(miss)) {
    if (miss) lsq_factor(m, X, f);
  }
  slope = 0.0;
  icpt = 0.0;
  ssr = 0.0;
  return act ? lsq_apply(f, X, Y, need_solution, need_ssr, slope, icpt, ssr) : 0;
}

// The vertex fits' least squares (solution only), in lockstep: one x-set lookup (lsq_factor for
// the lanes that miss), then the straight-line lsq_apply_small for the lanes whose segment has
// 2-4 points — nearly all of them — and the general lsq_apply for the rare longer ones, a branch
// the wave takes only if some lane needs it.
template <class GX, class GY>
__device__ inline int lsq_fit_lockstep(bool act, int m, GX X, GY Y,
                                       const lsq_xf* __restrict__ xtab, double& slope,
                                       double& icpt) {
  const int key = act ? xset_key(m, X) : 0;
  const bool miss = act && key < 0;
  lsq_xf f;
  if (act && !miss) f = xtab[key];
  if (__ballot(miss)) {
    if (miss) lsq_factor(m, X, f);
  }
  slope = 0.0;
  icpt = 0.0;
  int rc = 0;
  const bool big = act && m > 4;
  if (__ballot(big)) {
    if (big) {
      double ssr;
      rc = lsq_apply(f, X, Y, true, false, slope, icpt, ssr);
    }
  }
  if (act && m <= 4) rc = lsq_apply_small(f, X, Y, slope, icpt);
  return rc;
}

// VT: storage type of the series. The analyze stage stores int16 (an int16 index raster), binary32
// (other index types: pixels whose values are not exact in binary32 are sent to the resolve stage)
// or binary64 (binary64 values, up to 4 rules); the resolve stage the same, or binary64.
// AGLDS: the DP argmin of each column in LDS (resolve stage: its registers are spent on the exact
// DP) or, when false, in the lane's registers / private memory (analyze stage: 2 KB less LDS per
// wave, 15 instead of 12 resident waves per CU)
template <int MAXY, class VT, bool AGLDS>
struct WaveLds {
  VT ys[MAXY][64];       // present values (t), compacted in place to non-spike (k)
  uint8_t xn[MAXY][64];  // year offset of non-spike point k
  uint8_t ag[AGLDS ? MAXY : 1][64];  // DP argmin of column k (AGLDS only)
  int32_t year[LT_MAX_YEARS];  // the scene's calendar year per slot (64 words: one bank each)
};

// EXACT = false (analyze stage): the lazy DP; returns kDeferExact when the pixel's optimal path
// crosses an ambiguous DP column, kDeferWide when its values are not exact in binary32 (the
// resolve stage redoes them with binary32 / binary64 LDS series), else kDone.
// EXACT = true (resolve stage): the same lazy DP, but a column its intervals cannot decide is
// decided on the spot with the emulated LAPACK residuals of the candidates (and of the links of
// their optimal prefixes whose values are not yet exact); always kDone. (LT_RESOLVE_FULL: the
// exact-OPT DP over every column instead.)
enum { kDone = 0, kDeferExact = 1, kDeferWide = 2 };

// Phase probe of analyze_fast: probe.mark(k) is called by every lane at the end of phase k
// (0 winner pick, 1 despike, 2 DP, 3 vertex fits + per-year walk + rule offers, 4 label writes),
// and a probe whose kStopAfter is k ends the pixel there. The product kernels pass NoProbe (mark
// compiles to nothing, kStopAfter = -1 removes the exits); the profiling builds of profiles/
// (stamps.sh: cycle stamps; phases.sh: PMC counts of the kernel cut after each phase) define the
// others.
struct NoProbe {
  static constexpr int kStopAfter = -1;
  __device__ void mark(int) const {}
};

template <int MAXY, int RMAX, bool EXACT, class VT, class Probe = NoProbe>
__device__ inline int analyze_fast(const DevScene& S_launch, const lt_params& P, const lt_tile_in& in,
                                   const lt_tile_out& out, const lsq_xf* __restrict__ xtab,
                                   uint64_t* __restrict__ yflags, uint64_t* __restrict__ tl_bits,
                                   double* __restrict__ tl_eqn, int64_t p, bool live, int lane,
                                   WaveLds<MAXY, VT, EXACT>& L,
                                   const Probe& probe = Probe()) {
  // the scene: constants of a JIT kernel specialised for it (lt_jit.h), else the launch's
#ifdef LT_SPEC_SCENE
  const DevScene& S = lt_spec_scene;
  (void)S_launch;
#else
  const DevScene& S = S_launch;
#endif
#ifdef LT_SPEC_Y
  constexpr int Y = LT_SPEC_Y;
#else
  const int Y = S.n_years;
#endif
  const int64_t is = in.stride, os = out.stride;
  const double nan = __builtin_nan("");
  int status = LT_ST_OK;
  static_assert(LT_MAX_YEARS == 64, "one year-table word per lane");
  if (lane < Y) L.year[lane] = S.year[lane];
#ifdef LT_DEBUG_LDS_POISON
  // debugging (LT_JIT_DEFINES=LT_DEBUG_LDS_POISON=v): the lane's series slots filled with a junk
  // pattern first, so a read of a slot this pixel did not write shows up as a changed result
  for (int k = 0; k < MAXY; k++) {
    L.ys[k][lane] = (VT)(LT_DEBUG_LDS_POISON + 37 * k);
    L.xn[k][lane] = (uint8_t)(LT_DEBUG_LDS_POISON + 11 * k);
  }
#endif
  __syncthreads();  // one wave per workgroup: orders the table writes before any lane reads

  // ---- pick_winners (utils.py:491-521) over wave-uniform year slots ----
  int T = 0, y0 = 0;
  uint64_t pres = 0;  // year slots with a winner: present point t is the t-th set bit
  // int16 series: the values are integers of int16 range, so despike's standard deviation is
  // compared through the exact sums S = sum v, Q = sum v^2 (see the despike below)
  constexpr bool kIntSeries = std::is_same<VT, int16_t>::value;
  // a JIT kernel specialised for labels-only launches takes the branch-free store loop below (in
  // the per-year-output instances the same loop measured 1 % slower, profiles/r05_run29)
#if defined(LT_SPEC_YEAR_OUT) && LT_SPEC_YEAR_OUT == 0
  constexpr bool kFlatPick = true;
#else
  constexpr bool kFlatPick = false;
#endif
  double Ssum = 0.0, Qsum = 0.0;
  bool f32_bad = false;
  bool intdata = true;  // every value an integer of int16 range (lt_pixel.h sse_exact_zero)
  bool infdata = false;  // some value infinite (a binary32 series): the emulated fits fail (rc < 0)
  // years in batches of 8: the winners first, then their 8 value loads issued together (one
  // load per year in sequence would leave each wave waiting out the HBM latency 30 times)
  constexpr int WB = LT_WB;
  // the mask as bit planes (lt_tile_in.obs_valid_bits): up to 128 observations, the pixel's
  // words are loaded once, together, and the winner scan tests bits; a byte mask costs a load
  // per observation, each waited out before its year's comparison
#ifdef LT_SPEC_MASKED
  constexpr bool masked = LT_SPEC_MASKED != 0;
#ifdef LT_SPEC_VBITS
  // the mask's format as a constant (lt_jit.h Spec::vbits): one of the two scans is compiled
  constexpr bool vbits = masked && LT_SPEC_VBITS != 0;
#else
  const bool vbits = masked && in.obs_valid_bits != nullptr && S.n_obs <= 128;
#endif
#else
  const bool masked = in.obs_valid != nullptr || in.obs_valid_bits != nullptr;  // launch-uniform
  const bool vbits = in.obs_valid_bits != nullptr && S.n_obs <= 128;
#endif
  uint32_t vw0 = 0, vw1 = 0, vw2 = 0, vw3 = 0;
  if (vbits) {
    const uint32_t* vb = in.obs_valid_bits;
    const int64_t pq = live ? p : 0;
    const int nw = (S.n_obs + 31) >> 5;
    vw0 = vb[pq];
    if (nw > 1) vw1 = vb[is + pq];
    if (nw > 2) vw2 = vb[2 * is + pq];
    if (nw > 3) vw3 = vb[3 * is + pq];
  }
  for (int yb = 0; yb < Y; yb += WB) {
    int best[WB];
#pragma unroll
    for (int u = 0; u < WB; u++) {
      const int y = yb + u;
      best[u] = -1;
      if (y >= Y) continue;  // wave-uniform
      if (!masked) {  // launch-uniform: no mask, the scene's winner
        best[u] = live ? S.winner_all[y] : -1;
        continue;
      }
      int bd = 0x7fffffff;
      const int k1 = S.slot_begin[y + 1];
      for (int k = S.slot_begin[y]; k < k1; k++) {
        const int o = S.order[k];
        bool ok;
        if (vbits) {  // o is wave-uniform: a scalar choice of the word
          const uint32_t wd = o < 32 ? vw0 : o < 64 ? vw1 : o < 96 ? vw2 : vw3;
          ok = live && ((wd >> (o & 31)) & 1u);
        } else {
          ok = live && obs_is_valid(in, o, p);
        }
        if (ok && S.dist[k] < bd) {
          bd = S.dist[k];
          best[u] = o;
        }
      }
    }
    double val[WB];
    // Loads of the batch: unconditional (obs 0 / pixel 0 stand in), all WB in flight at once, one
    // typed batch per launch-uniform type. Without a cloud mask every lane's winner of a year is
    // the scene's (uniform: UNI), so a load is the row's base in SGPRs plus the lane's 32-bit
    // offset — no per-lane 64-bit address arithmetic; with a mask each lane has its own row.
    const uint32_t pp = live ? (uint32_t)p : 0u;  // pixel offset within a row
    __builtin_assume(pp < (1u << 28));             // tiles hold <= LT_MAX_TILE_PIX pixels
    auto row_of = [&](int u, auto uni) -> int64_t {
      if constexpr (decltype(uni)::value) {
        const int w = yb + u < Y ? S.winner_all[yb + u] : 0;
        return w > 0 ? w : 0;
      } else {
        return best[u] >= 0 ? best[u] : 0;
      }
    };
    auto batch = [&](auto tag, auto uni) {
      using T = decltype(tag);
      const T* base = in.obs_index ? (const T*)in.obs_index : (const T*)in.obs_val;
      T raw[WB];
#pragma unroll
      for (int u = 0; u < WB; u++) raw[u] = (base + row_of(u, uni) * is)[pp];
#pragma unroll
      for (int u = 0; u < WB; u++) val[u] = (double)raw[u];
    };
    // the fused load stage (lt_abi.h lt_index_lin) for int16 bands and a narrow form (node type
    // of <= 32 bits, coefficients of 24 bits; 'B1 - B2'): the winners' band values, every load of
    // the batch in flight at once, then 32-bit arithmetic — a multiply-add per band, one wrap, one
    // clamp, one conversion (the sum is needed only modulo 2^bits(node type) <= 2^32). Other forms
    // take obs_value's general path (lt_pixel.h lin_value), one value at a time: one instance of
    // the batch keeps the kernel's code and register allocation as they are without it
    auto fused16 = [&](auto uni) {
      const lt_index_lin& LN = in.lin;
      const int nb = LN.n_bands;
      int32_t acc[WB];  // the sum modulo 2^32: a 24-bit multiply-add per band
      // a pixel-interleaved pair: one 32-bit load (check_tile: 4-byte aligned, even obs stride).
      // A planar tile of one pixel may also have band_stride 1: not a pair
      if (nb == 2 && in.band_stride == 1 && in.band_pix_stride == 2) {
        const int32_t* bw = (const int32_t*)in.obs_bands;
        const int64_t os2 = in.band_obs_stride >> 1;
        int32_t w[WB];
#pragma unroll
        // nontemporal: the band pairs are read once; the x-set table stays L2-hot (c5 +1.4 %,
        // profiles/r03_ab13)
        for (int u = 0; u < WB; u++)
          w[u] = __builtin_nontemporal_load(&(bw + row_of(u, uni) * os2)[pp]);
        const int c0 = (int)(uint32_t)LN.c0, k0 = (int)LN.coef[0], k1 = (int)LN.coef[1];
#pragma unroll
        for (int u = 0; u < WB; u++) {
          // band plane 0 at the lower address (the builtin returns unsigned: the cast keeps the
          // sign-extended bits)
          const int b0 = (int32_t)__builtin_amdgcn_sbfe(w[u], 0, 16), b1 = w[u] >> 16;
          acc[u] = __mul24(k1, b1) + (__mul24(k0, b0) + c0);
        }
      } else {
        const int16_t* bb = (const int16_t*)in.obs_bands;
#pragma unroll
        for (int u = 0; u < WB; u++) acc[u] = (int32_t)(uint32_t)LN.c0;
#pragma unroll
        for (int s = 0; s < LT_LIN_MAX_BANDS; s++) {
          if (s >= nb) break;  // launch-uniform
          int16_t raw[WB];
#pragma unroll
          for (int u = 0; u < WB; u++)
            raw[u] = bb[row_of(u, uni) * in.band_obs_stride + s * in.band_stride +
                        (int64_t)pp * in.band_pix_stride];
#pragma unroll
          for (int u = 0; u < WB; u++) acc[u] = __mul24((int)LN.coef[s], (int)raw[u]) + acc[u];
        }
      }
      const int wb = lin_type_bits(LN.wrap_type);
      const bool sgn = lin_type_signed(LN.wrap_type);
      int64_t lo64, hi64, wlo, whi;
      lin_out_range(LN.out_type, lo64, hi64);
      lin_out_range(LN.wrap_type, wlo, whi);
      // launch-uniform fast case ('B1 - B2': int16 nodes stored as int16 or binary64): a signed
      // wrap (one bit-field extract, none for 32 bits) into a store type that holds every wrapped
      // value, so the clamp is the identity, and an exact conversion
      if (sgn && lo64 <= wlo && hi64 >= whi && LN.out_type != LT_T_F32) {
        if (wb < 32) {
#pragma unroll
          for (int u = 0; u < WB; u++) val[u] = (double)(int32_t)__builtin_amdgcn_sbfe(acc[u], 0, wb);
        } else {
#pragma unroll
          for (int u = 0; u < WB; u++) val[u] = (double)acc[u];
        }
        return;
      }
      const int sh = 32 - wb;
      const int32_t lo = lo64 < INT32_MIN ? INT32_MIN : (int32_t)lo64;
      const int32_t hi = hi64 > INT32_MAX ? INT32_MAX : (int32_t)hi64;
#pragma unroll
      for (int u = 0; u < WB; u++) {
        const uint32_t a = (uint32_t)acc[u];
        const int32_t r = sgn ? (int32_t)(a << sh) >> sh : (int32_t)((a << sh) >> sh);
        if (LN.out_type == LT_T_F64) val[u] = (double)r;
        else if (LN.out_type == LT_T_F32) val[u] = (double)(float)r;
        else val[u] = (double)(r < lo ? lo : r > hi ? hi : r);
      }
    };
    using Uni = std::true_type;
    using Lane = std::false_type;
    const bool uni = !masked;  // launch-uniform
#ifdef LT_JIT_INDEX
    // a JIT kernel (lt_jit.h): the tile's index_eqn program is inlined as lt_jit_index (the load
    // kernel's straight-line code and store, lt_index.h codegen), evaluated on every winner's
    // band values, all the batch's band loads issued first
#if defined(LT_SPEC_BAND_PAIR) && LT_SPEC_BAND_PAIR
    {
      // two 16-bit bands pixel-interleaved, 4-byte aligned (lt_jit.h Spec::band_pair): a pixel's
      // pair is one 32-bit load, nontemporal (read once; the x-set table stays L2-hot), band 0 in
      // the low half, as the fused linear path reads it (fused16)
      const int32_t* bw = (const int32_t*)in.obs_bands;
      const int64_t os2 = in.band_obs_stride >> 1;
      int32_t w[WB];
#pragma unroll
      for (int u = 0; u < WB; u++)
        w[u] = __builtin_nontemporal_load(
            &(bw + (uni ? row_of(u, Uni{}) : row_of(u, Lane{})) * os2)[pp]);
#pragma unroll
      for (int u = 0; u < WB; u++) {
        const LT_JIT_BAND_T b2[2] = {(LT_JIT_BAND_T)(w[u] & 0xffff),
                                     (LT_JIT_BAND_T)((uint32_t)w[u] >> 16)};
        val[u] = lt_jit_index(b2, 1);
      }
    }
#else
    {
      const LT_JIT_BAND_T* bb = (const LT_JIT_BAND_T*)in.obs_bands;
      const LT_JIT_BAND_T* at[WB];
#pragma unroll
      for (int u = 0; u < WB; u++)
        at[u] = bb + (uni ? row_of(u, Uni{}) : row_of(u, Lane{})) * in.band_obs_stride +
                (int64_t)pp * in.band_pix_stride;
#pragma unroll
      for (int u = 0; u < WB; u++) val[u] = lt_jit_index(at[u], in.band_stride);
    }
#endif
#else
    if (in.obs_bands) {
      const lt_index_lin& LN = in.lin;
      const int wb = lin_type_bits(LN.wrap_type);
      bool narrow = LN.band_type == LT_T_I16 && wb <= 32 &&
                    (wb < 32 || lin_type_signed(LN.wrap_type));
#pragma unroll
      for (int s = 0; s < LT_LIN_MAX_BANDS; s++)
        if (s < LN.n_bands) narrow = narrow && LN.coef[s] >= -(1 << 23) && LN.coef[s] < (1 << 23);
      if (narrow) {
        if (uni) fused16(Uni{});
        else fused16(Lane{});
      } else {
#pragma unroll
        for (int u = 0; u < WB; u++)
          val[u] = obs_value(in, (int64_t)(best[u] >= 0 ? best[u] : 0), live ? p : 0);
      }
    } else if (in.obs_index == nullptr) {
      if (uni) batch(double{}, Uni{});
      else batch(double{}, Lane{});
    } else if (in.index_type == LT_T_I16) {
      if (uni) batch(int16_t{}, Uni{});
      else batch(int16_t{}, Lane{});
    } else if (in.index_type == LT_T_F32) {
      batch(float{}, Lane{});
    } else if (in.index_type == LT_T_U16) {
      batch(uint16_t{}, Lane{});
    } else if (in.index_type == LT_T_I32) {
      batch(int32_t{}, Lane{});
    } else if (in.index_type == LT_T_U8) {
      batch(uint8_t{}, Lane{});
    } else {
#pragma unroll
      for (int u = 0; u < WB; u++)
        val[u] = obs_value(in, (int64_t)(best[u] >= 0 ? best[u] : 0), live ? p : 0);
    }
#endif  // LT_JIT_INDEX
#pragma unroll
    for (int u = 0; u < WB; u++) {
      const int y = yb + u;
      if (y >= Y) break;  // wave-uniform
      if constexpr (kIntSeries && kFlatPick) {
        // labels-only int16 series, branch-free: every lane takes the step; a lane without the
        // year (or dead) writes slot T (its next point overwrites it; past its series it is never
        // read) and keeps T and the sums (c2 +1.4 %, c3 +1.1 %, profiles/r05_run29)
        if (!LT_OUTF(out, winner) && !LT_OUTF(out, val_raw)) {  // launch-uniform
          const bool pr = live && best[u] >= 0;
          if ((S.feb29_mask >> y) & 1) status |= pr ? LT_ST_FEB29 : 0;
          const double v = val[u];
          const int ty = S.year[y];
          y0 = (pr && T == 0) ? ty : y0;
          L.ys[T][lane] = (VT)v;
          L.xn[T][lane] = (uint8_t)(ty - y0);
          const double vp = pr ? v : 0.0;
          Ssum += vp;
          Qsum = __builtin_fma(vp, vp, Qsum);
          pres |= pr ? 1ull << y : 0ull;
          T += pr ? 1 : 0;
          continue;
        }
      }
      if (!live) continue;
      const int64_t q = (int64_t)y * os + p;
      if (LT_OUTF(out, winner) && LT_AB_NO_YEAR_STORES < 2)
        __builtin_nontemporal_store((int16_t)best[u], LT_OUTF(out, winner) + q);
      if (best[u] >= 0) {
        if ((S.feb29_mask >> y) & 1) status |= LT_ST_FEB29;
        const double v = val[u];
        if (T == 0) y0 = S.year[y];
        const VT vs = (VT)v;
        // (an int16 series holds int16 index values, stored or evaluated: always exact)
        if constexpr ((!EXACT || sizeof(VT) < 8) && !kIntSeries) {
          if (!((double)vs == v)) f32_bad = true;
        }
        if constexpr (!std::is_same<VT, int16_t>::value) {
          if (!(v == __builtin_rint(v) && __builtin_fabs(v) <= 32767.0)) intdata = false;
          if (__builtin_isinf(v)) infdata = true;
        }
        L.ys[T][lane] = vs;
        if constexpr (kIntSeries) {
          // the point's year offset (the scan below compacts it with its value) and the exact
          // sums: integers below 2^53
          L.xn[T][lane] = (uint8_t)(S.year[y] - y0);
          Ssum += v;
          Qsum = __builtin_fma(v, v, Qsum);
        }
        pres |= 1ull << y;
        T++;
        if (LT_OUTF(out, val_raw) && LT_AB_NO_YEAR_STORES < 2)
          year_row_store(v, LT_OUTF(out, val_raw) + q);
      } else if (LT_OUTF(out, val_raw) && LT_AB_NO_YEAR_STORES < 2) {  // the other per-year planes: the year-major output loop
        __builtin_nontemporal_store(nan, LT_OUTF(out, val_raw) + q);
      }
    }
  }
  probe.mark(0);
  if constexpr (Probe::kStopAfter == 0) return kDone;
  // the reference raises for T < 2; non-binary32 values take the resolve stage's double path
  const bool ok = live && T >= 2 && !f32_bad;
  if (live && T == 0) status |= LT_ST_EMPTY;
  if (live && T == 1) status |= LT_ST_SINGLE_YEAR;
  const int Tmax = wave_max(ok ? T : 0);

  // ---- despike (utils.py:556-582): numpy pairwise std, then the 3-window scan ----
  uint64_t spike = 0;
  int n = 0;
  if (kIntSeries && Tmax >= 2) {
    // int16 series. The reference's sd is numpy's (pairwise sums of v and of (avg - v)^2, below
    // in the general path); its only use is the test |y - x| > sd on an integer |y - x| <= 2^16.
    // In exact arithmetic sd^2 = N / T^2 with N = T Q - S^2 (an integer < 2^43, exact here), so
    // |d| > sd_exact <=> d^2 T^2 > N <=> |d| >= K, K = the least integer a with a^2 T^2 > N.
    // numpy's sd is within 11.5 ulp (2^-49.5, relative) of sd_exact (pairwise sums of <= 64
    // positive terms: <= 17 roundings on any term's path; avg's rounding only adds T (avg -
    // S/T)^2 <= 2^-70 N/T), while an integer a <= 2^16 that is not sd_exact lies at least
    // 1 / (2 a T^2) >= 2^-45 a from it (a^2 T^2 - N is a nonzero integer): the two tests agree
    // for every |d| except |d| = sd_exact, an integer. Such a lane (N = a^2 T^2) takes numpy's
    // sd (the pairwise sums, ballot-gated) to decide whether |d| = a counts as above it.
    const double Td = (double)T, T2 = Td * Td;
    const double N = __builtin_fma(Td, Qsum, -(Ssum * Ssum));
    double a = ok ? __builtin_floor((double)__builtin_sqrtf((float)N) / Td) : 0.0;  // +-1
    if (a * a * T2 > N) a -= 1.0;
    if ((a + 1.0) * (a + 1.0) * T2 <= N) a += 1.0;
    int K = (int)a + 1;  // |d| > sd <=> |d| >= K
    const bool tie = ok && a * a * T2 == N;
    if (__ballot(tie)) {
      // numpy's sd for the lanes whose exact sd is the integer a: sequential-over-blocks
      // pairwise sums as the general path computes them (np.sum)
      const int n8 = (tie && T >= 8) ? T - (T % 8) : 0;
      auto npsum = [&](auto term) {
        double r[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        for (int t0 = 0; t0 < n8; t0 += 8)
          for (int u = 0; u < 8; u++) r[u] = t0 == 0 ? term(u) : r[u] + term(t0 + u);
        double seq = n8 > 0 ? ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
                            : 0.0;
        for (int t = n8; t < T; t++) seq += term(t);
        return seq;
      };
      if (tie) {
        const double avg = npsum([&](int t) { return (double)L.ys[t][lane]; }) / Td;
        const double sd = __builtin_sqrt(npsum([&](int t) {
                                           const double d = avg - (double)L.ys[t][lane];
                                           return d * d;
                                         }) /
                                         Td);
        if (a > sd) K = (int)a;
      }
    }
    // the 3-window scan in int32 (the values are exact), fused with dropna's compaction of the
    // values and of the year offsets the winner pick stored (slot n <= t is written once point
    // t's decision is known; this block's reads come first)
    int last_good = ok ? (int)L.ys[0][lane] : 0;
    int xv = last_good, yv = ok ? (int)L.ys[1][lane] : 0;
    if (ok) n = 1;  // point 0 is never a spike (its offset, 0, is in place)
    const int nK = -K;
    for (int t0 = 1; t0 < Tmax; t0 += 8) {
      int z[8], xo[8];
      // unconditional LDS reads (the slot index clamped into the arrays; a value past the
      // lane's T is never used): a guarded read per slot cost a scalar branch and a
      // condition moved through a VGPR each
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int tz = t0 + u + 1 < MAXY ? t0 + u + 1 : MAXY - 1;
        const int tx = t0 + u < MAXY ? t0 + u : MAXY - 1;
        z[u] = (int)L.ys[tz][lane];
        xo[u] = (int)L.xn[tx][lane];
      }
      // branch-free per point: every lane takes every step (a lane past its last point, or
      // without one, only rewrites the slot past its compacted series and keeps n), so the wave
      // runs no exec-mask juggling per point; the last point is never a spike (mid)
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int t = t0 + u;
        if (t >= Tmax) break;  // wave-uniform
        const bool inr = ok && t < T;  // the lane has point t
        const int cur = yv;
        const int zv = z[u];
        const int d1 = yv - xv, d2 = zv - yv;
        // not monotone (x <= y <= z or x >= y >= z fails: the steps have strictly opposite
        // signs) with both |steps| >= K: as K >= 1, one step >= K and the other <= -K
        const bool big = (d1 >= K && d2 <= nK) || (d1 <= nK && d2 >= K);
        const bool is_spike = inr && t + 1 < T && big && yv != last_good;
        last_good = is_spike ? last_good : yv;  // (a lane past its points never reads it)
        xv = yv;
        yv = zv;
        spike |= is_spike ? (1ull << t) : 0ull;
        // slot n gets point t; n moves on for a kept point (slot n = t before the first spike:
        // the same values rewritten)
        L.ys[n][lane] = (VT)cur;
        L.xn[n][lane] = (uint8_t)xo[u];
        n += (inr && !is_spike) ? 1 : 0;
      }
    }
  } else if (Tmax >= 2) {
    // np.sum: n >= 8: eight accumulators over the first n - n%8 elements
    // (r_k starts as element k), their tree, then the rest sequentially; n < 8: sequential.
    // Two uniform loops: the accumulator block up to the wave's largest n8, the sequential tail
    // from the wave's smallest n8 (per-lane predicates select which elements a lane takes).
    const int n8 = (ok && T >= 8) ? T - (T % 8) : 0;
    const int n8max = wave_max(n8);
    const int n8min = -wave_max(-n8);
    // elements are read eight at a time (eight LDS reads in flight, then the adds)
    auto npsum = [&](auto term) {
      double r0 = 0.0, r1 = 0.0, r2 = 0.0, r3 = 0.0, r4 = 0.0, r5 = 0.0, r6 = 0.0, r7 = 0.0;
      for (int t0 = 0; t0 < n8max; t0 += 8) {  // t0 wave-uniform, t0 + 7 < n8max <= MAXY
        const bool in = t0 < n8;
        double a[8];
#pragma unroll
        for (int u = 0; u < 8; u++) a[u] = term(t0 + u);
        if (t0 == 0) {  // r_k starts as element k
          r0 = a[0]; r1 = a[1]; r2 = a[2]; r3 = a[3];
          r4 = a[4]; r5 = a[5]; r6 = a[6]; r7 = a[7];
        } else if (in) {
          r0 = r0 + a[0]; r1 = r1 + a[1]; r2 = r2 + a[2]; r3 = r3 + a[3];
          r4 = r4 + a[4]; r5 = r5 + a[5]; r6 = r6 + a[6]; r7 = r7 + a[7];
        }
      }
      double seq = n8 > 0 ? ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) : 0.0;
      for (int t0 = n8min; t0 < Tmax; t0 += 8) {
        double a[8];
#pragma unroll
        for (int u = 0; u < 8; u++) a[u] = t0 + u < Tmax ? term(t0 + u) : 0.0;  // uniform guard
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const int t = t0 + u;
          if (ok && t >= n8 && t < T) seq += a[u];  // sequential, in element order
        }
      }
      return seq;
    };
    const double avg = npsum([&](int t) { return L.ys[t][lane]; }) / (double)T;
    const double sd = __builtin_sqrt(npsum([&](int t) {
                                       const double d = avg - L.ys[t][lane];
                                       return d * d;
                                     }) /
                                     (double)T);
    // the 3-window scan (on the original series) fused with dropna's in-place compaction: point
    // t is written to slot n <= t once its spike decision is known; ys[t + 1] is read first
    uint64_t rem = pres;
    double last_good = ok ? L.ys[0][lane] : 0.0;
    double xv = last_good, yv = ok ? L.ys[1][lane] : 0.0;
    if (ok) {  // point 0 is never a spike
      const int y = __builtin_ctzll(rem);
      rem &= rem - 1;
      L.xn[0][lane] = (uint8_t)(L.year[y] - y0);
      n = 1;
    }
    for (int t0 = 1; t0 < Tmax; t0 += 8) {
      // the next eight right neighbours first (eight LDS reads in flight); this block's writes
      // go to slots <= t0 + 7, all read already
      double z[8];
#pragma unroll
      for (int u = 0; u < 8; u++) z[u] = t0 + u + 1 < Tmax ? (double)L.ys[t0 + u + 1][lane] : 0.0;
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int t = t0 + u;
        if (t >= Tmax) break;  // wave-uniform
        if (!(ok && t < T)) continue;
        const double cur = yv;  // ys[t]
        bool is_spike = false;
        if (t + 1 < T) {  // the last point is never a spike
          const double zv = z[u];
          const bool mono = (xv <= yv && yv <= zv) || (xv >= yv && yv >= zv);
          is_spike = !mono && (__builtin_fabs(yv - xv) > sd && __builtin_fabs(yv - zv) > sd) &&
                     yv != last_good;
          if (!is_spike) last_good = yv;
          xv = yv;
          yv = zv;
        }
        const int y = __builtin_ctzll(rem);
        rem &= rem - 1;
        if (is_spike) {
          spike |= 1ull << t;
          continue;
        }
        if (n != t) L.ys[n][lane] = (VT)cur;
        L.xn[n][lane] = (uint8_t)(L.year[y] - y0);
        n++;
      }
    }
  }
  probe.mark(1);
  if constexpr (Probe::kStopAfter == 1) return kDone;
  const int nmax = wave_max(n);

  // ---- segmented least squares DP (utils.py:618-631), decided lazily ----
  bool deferred = live && T >= 2 && f32_bad;
  uint64_t vmask = 0;  // vertices over non-spike indices
  // DP argmin of each column (see WaveLds): written at wave-uniform columns, read once per vertex
  // by the backtrack
  uint8_t AG[EXACT ? 1 : MAXY];
  auto ag_set = [&](int j, int a) {
    if constexpr (EXACT) L.ag[j][lane] = (uint8_t)a;
    else AG[j] = (uint8_t)a;
  };
  auto ag_get = [&](int j) -> int {
    if constexpr (EXACT) return L.ag[j][lane];
    else return AG[j];
  };
  if constexpr (EXACT && LT_RESOLVE_FULL != 0) {
    if constexpr (MAXY <= LT_RESOLVE_PRIV_MAXY) {
      // ---- exact-OPT DP: closed-form intervals, then the emulated LAPACK residual for every
      // start whose interval reaches the column's smallest upper bound; first exact minimum ----
      const double c = LT_LINE_COST;
      const double inf = __builtin_inf();
      // OPT lives in per-lane private memory (read at wave-uniform and per-lane indices)
      double OPT[MAXY + 1];
      OPT[0] = 0.0;
      double SyyAll = 0.0;  // sum of y^2 over the points 0..j (early-exit bound, as below)
      const bool prune = c >= 0.0;
      for (int jj = 0; jj < nmax; jj++) {
        const int j = __builtin_amdgcn_readfirstlane(jj);
        const bool col = j < n;
        double Sy = 0.0, Sxy = 0.0, Syy = 0.0;
        int Sx = 0, Sxx = 0;
        double H = inf;
        // starts whose interval reaches the smallest upper end seen so far (itself included): a
        // superset of those reaching the final one, where the exact minimum lies
        uint64_t cand = 0;
        {
          const double yj = (double)L.ys[j][lane];
          SyyAll = __builtin_fma(yj, yj, SyyAll);
        }
        // the next start's operands are loaded one iteration ahead, so the LDS and private-memory
        // latency overlaps this start's arithmetic
        int xpre = L.xn[j][lane];
        VT ypre = L.ys[j][lane];
        double opre = OPT[j];
        for (int ii = j; ii >= 0; ii--) {
          const int i = __builtin_amdgcn_readfirstlane(ii);  // wave-uniform start
          const int xi = xpre;
          const double yi = (double)ypre;
          const double oi = opre;
          if (i > 0) {
            xpre = L.xn[i - 1][lane];
            ypre = L.ys[i - 1][lane];
            opre = OPT[i - 1];
          }
          Sx += xi;
          Sxx += xi * xi;
          Sy += yi;
          Sxy = __builtin_fma((double)xi, yi, Sxy);
          Syy = __builtin_fma(yi, yi, Syy);
          const int m = j - i + 1;
          double e = 0.0, w = 0.0;  // m <= 2: exact residual 0 on an exact OPT: v is the reference
          if (m >= 3) {
            const double md = (double)m;
            const double D = (double)(m * Sxx - Sx * Sx);
            const double t1 = __builtin_fma(md, Syy, -(Sy * Sy));
            const double N1 = __builtin_fma(md, Sxy, -((double)Sx * Sy));
            const double den = md * D;
            double r = __builtin_amdgcn_rcp(den);
            r = __builtin_fma(r, __builtin_fma(-den, r, 1.0), r);
            e = __builtin_fma(t1, D, -(N1 * N1)) * r;
            e = e < 0.0 ? 0.0 : e;
          }
          const double v = (e + c) + oi;
          if (m >= 3) w = __builtin_fma(0x1p-50, __builtin_fabs(v), kScreen * Syy);
          if (v - w <= H) cand |= 1ull << i;
          H = v + w < H ? v + w : H;
          // early exit (dp_start_bound): no start below i can reach H
          if (prune && m >= 3 && !__ballot(col && !(dp_start_bound(e, oi, 0.0, c, SyyAll) > H)))
            break;
        }
        const int nc = col ? __builtin_popcountll(cand) : 0;
        const int ncmax = wave_max(nc);
        double best = inf;
        int bi = 0;
        for (int r = 0; r < ncmax; r++) {  // candidates in increasing start order, lockstep
          const bool act = r < nc;
          const int i = act ? __builtin_ctzll(cand) : 0;
          if (act) cand &= cand - 1;
          const double oi = OPT[i];  // per-lane index, loaded before the fit that hides it
          const int m = j - i + 1;
          const bool ls = act && m >= 3;
          double e = 0.0;
          if (__ballot(ls)) {
            double sm, sb, ssr;
            const int rc = lsq_lockstep(
                ls, m, [&](int k) { return (int)L.xn[i + k][lane]; },
                [&](int k) { return (double)L.ys[i + k][lane]; }, xtab, false, true, sm, sb, ssr);
            if (ls) {
              if (rc < 0) status |= LT_ST_NUMERIC;
              e = ssr;
            }
          }
          const double v = (e + c) + oi;
          if (act && v < best) {  // increasing start order + strict "<": the first minimum
            best = v;
            bi = i;
          }
        }
        if (col) {
          ag_set(j, bi);
          OPT[j + 1] = best;
        }
      }
    } else {  // larger series: OPT in registers (private memory would thrash L1)
      // ---- exact-OPT DP: closed-form intervals, then the emulated LAPACK residual for every
      // start whose interval reaches the column's smallest upper bound; first exact minimum ----
      const double c = LT_LINE_COST;
      const double inf = __builtin_inf();
      double OPT[MAXY + 1];
#pragma unroll
      for (int k = 0; k <= MAXY; k++) OPT[k] = 0.0;
      double SyyAll = 0.0;  // sum of y^2 over the points 0..j (early-exit bound, as below)
      const bool prune = c >= 0.0;
      for (int jj = 0; jj < nmax; jj++) {
        const int j = __builtin_amdgcn_readfirstlane(jj);
        const bool col = j < n;
        double Sy = 0.0, Sxy = 0.0, Syy = 0.0;
        int Sx = 0, Sxx = 0;
        double H = inf;
        // starts whose interval reaches the smallest upper end seen so far (itself included): a
        // superset of those reaching the final one, where the exact minimum lies
        uint64_t cand = 0;
        {
          const double yj = (double)L.ys[j][lane];
          SyyAll = __builtin_fma(yj, yj, SyyAll);
        }
#pragma unroll
        for (int i = MAXY - 1; i >= 0; i--) {
          if (i > j) continue;  // wave-uniform
          const int xi = L.xn[i][lane];
          const double yi = (double)L.ys[i][lane];
          Sx += xi;
          Sxx += xi * xi;
          Sy += yi;
          Sxy = __builtin_fma((double)xi, yi, Sxy);
          Syy = __builtin_fma(yi, yi, Syy);
          const int m = j - i + 1;
          double e = 0.0, w = 0.0;  // m <= 2: exact residual 0 on an exact OPT: v is the reference
          if (m >= 3) {
            const double md = (double)m;
            const double D = (double)(m * Sxx - Sx * Sx);
            const double t1 = __builtin_fma(md, Syy, -(Sy * Sy));
            const double N1 = __builtin_fma(md, Sxy, -((double)Sx * Sy));
            const double den = md * D;
            double r = __builtin_amdgcn_rcp(den);
            r = __builtin_fma(r, __builtin_fma(-den, r, 1.0), r);
            e = __builtin_fma(t1, D, -(N1 * N1)) * r;
            e = e < 0.0 ? 0.0 : e;
          }
          const double v = (e + c) + OPT[i];
          if (m >= 3) w = __builtin_fma(0x1p-50, __builtin_fabs(v), kScreen * Syy);
          if (v - w <= H) cand |= 1ull << i;
          H = v + w < H ? v + w : H;
          // early exit (dp_start_bound): no start below i can reach H
          if (prune && m >= 3 && !__ballot(col && !(dp_start_bound(e, OPT[i], 0.0, c, SyyAll) > H)))
            break;
        }
        const int nc = col ? __builtin_popcountll(cand) : 0;
        const int ncmax = wave_max(nc);
        double best = inf;
        int bi = 0;
        for (int r = 0; r < ncmax; r++) {  // candidates in increasing start order, lockstep
          const bool act = r < nc;
          const int i = act ? __builtin_ctzll(cand) : 0;
          if (act) cand &= cand - 1;
          const int m = j - i + 1;
          const bool ls = act && m >= 3;
          double e = 0.0;
          if (__ballot(ls)) {
            double sm, sb, ssr;
            const int rc = lsq_lockstep(
                ls, m, [&](int k) { return (int)L.xn[i + k][lane]; },
                [&](int k) { return (double)L.ys[i + k][lane]; }, xtab, false, true, sm, sb, ssr);
            if (ls) {
              if (rc < 0) status |= LT_ST_NUMERIC;
              e = ssr;
            }
          }
          double o = 0.0;
#pragma unroll
          for (int k = 0; k < MAXY; k++)
            if (k == i) o = OPT[k];  // per-lane index: select chain
          const double v = (e + c) + o;
          if (act && v < best) {  // increasing start order + strict "<": the first minimum
            best = v;
            bi = i;
          }
        }
        if (col) {
          ag_set(j, bi);
#pragma unroll
          for (int k = 1; k <= MAXY; k++)
            if (k == j + 1) OPT[k] = best;  // wave-uniform index
        }
      }
    }
    if (n >= 1) {
      vmask = 1ull << (n - 1);
      for (int j = n - 1; j >= 0;) {
        const int a = ag_get(j);
        vmask |= 1ull << a;
        j = a - 1;
      }
    }
  } else if (nmax >= 1) {
    const double c = LT_LINE_COST;
    const double inf = __builtin_inf();
    double OPTa[MAXY + 1];  // per-lane private memory (wave-uniform indices)
    OPTa[0] = 0.0;
    uint64_t exact = 1;      // bit k: OPTa[k] is the reference value itself
    double Emax = 0.0;       // bound on |OPTa[k] - OPT[k]| for every inexact k so far
    // register window of the four most recent points (x, y of points j..j-3) and of OPTa[j..j-3]:
    // the 1- to 4-point starts of a column, nearly all the DP prices, read no LDS or private
    // memory. Four register slots per quantity; the column loop is unrolled by four and each
    // column receives the slots rotated, so the window moves without register copies.
    int xA = 0, xB = 0, xC = 0, xD = 0;
    double yA = 0.0, yB = 0.0, yC = 0.0, yD = 0.0;
    double oA = 0.0, oB = 0.0, oC = 0.0, oD = 0.0;  // oA = OPTa[0] for column 0
    // tags of the OPTa window slots (lt_pixel.h tag_order; < 256: the value is exact)
    int gA = 0, gB = 0, gC = 0, gD = 0;
    double SyyAll = 0.0;                // sum of y^2 over the points 0..j
    const bool prune = c >= 0.0;
    // zero-residual starts of >= 3 points (lt_pixel.h kZero): integer series of int16 range only
    const bool zok = c > 0.0;
    const bool zlane = zok && intdata;
    const uint64_t zmask = __ballot(zlane);
    uint64_t amb = 0;
    // resolve stage: the exact decision of column j for the lanes xr (see column below). One
    // lockstep loop of emulated residuals: per lane first the links k (OPTa[k] = fl(fl(e(a, k-1) +
    // c) + OPTa[a]), a = argmin of column k-1) that the candidates' OPT values need, in increasing
    // k, then the candidates in increasing start order (strict "<": the first minimum)
    auto resolve_column = [&](const int j, const bool xr, const double H, uint64_t cs,
                              const double opt_j, const int tg_j, const double opt_jm1,
                              const int tg_jm1, int& a, double& vnew) {
      // the 1- and 2-point starts j, j-1 (residual 0), when their interval reaches H
      {
        const double v0 = c + opt_j;
        const double w0 = tg_j < 256 ? 0.0 : __builtin_fma(0x1p-50, __builtin_fabs(v0), Emax);
        if (!(v0 - w0 > H)) cs |= 1ull << j;
        if (j >= 1) {
          const double v1s = c + opt_jm1;
          const double w1 =
              tg_jm1 < 256 ? 0.0 : __builtin_fma(0x1p-50, __builtin_fabs(v1s), Emax);
          if (!(v1s - w1 > H)) cs |= 1ull << (j - 1);
        }
      }
      if (!xr) cs = 0;
      uint64_t need = cs & ~exact;  // OPTa entries to make exact, with their prefixes' links
      {
        const int top = wave_max(need ? 63 - __builtin_clzll(need) : 0);
        for (int kk = top; kk >= 1; kk--) {
          const int k = __builtin_amdgcn_readfirstlane(kk);
          if ((need >> k) & 1) {
            const int b = L.ag[k - 1][lane];
            if (!((exact >> b) & 1)) need |= 1ull << b;
          }
        }
      }
      const int steps = wave_max(__builtin_popcountll(need) + __builtin_popcountll(cs));
      double best = inf;
      int bi = 0;
      for (int r = 0; r < steps; r++) {
        const bool link = need != 0;
        const bool act = link || cs != 0;
        int i = 0, m = 0;  // the segment: points i .. i+m-1
        int k = 0;
        if (link) {
          k = __builtin_ctzll(need);
          need &= need - 1;
          i = L.ag[k - 1][lane];
          m = k - i;
        } else if (act) {
          i = __builtin_ctzll(cs);
          cs &= cs - 1;
          m = j - i + 1;
        }
        const bool ls = act && m >= 3;
        double e = 0.0;
        if (__ballot(ls)) {
          double sm, sb, ssr;
          const int rc = lsq_lockstep(
              ls, m, [&](int q) { return (int)L.xn[i + q][lane]; },
              [&](int q) { return (double)L.ys[i + q][lane]; }, xtab, false, true, sm, sb, ssr);
          if (ls) {
            if (rc < 0) status |= LT_ST_NUMERIC;
            e = ssr;
          }
        }
        if (act) {
          const double v = (e + c) + OPTa[i];  // per-lane index: exact by now
          if (link) {
            OPTa[k] = v;
            exact |= 1ull << k;
          } else if (v < best) {
            best = v;
            bi = i;
          }
        }
      }
      if (xr) {
        a = bi;
        vnew = best;
      }
    };
    // column j: wx0 receives point j (its slot held point j-4); wx1..wx3 hold points j-1..j-3;
    // opt_j..opt_jm3 hold OPTa[j..j-3] (tags tg_*), and OPTa[j+1] is written over opt_jm3
    auto column = [&](const int j, int& wx0, int& wx1, int& wx2, int& wx3, double& wy0,
                      double& wy1, double& wy2, double& wy3, double& opt_j, double& opt_jm1,
                      double& opt_jm2, double& opt_jm3, int& tg_j, int& tg_jm1, int& tg_jm2,
                      int& tg_jm3) __attribute__((always_inline)) {
      const bool col = j < n;
      const uint64_t colmask = __ballot(col);
      double Sy = 0.0, Sxy = 0.0, Syy = 0.0;
      int Sx = 0, Sxx = 0;
      // interval candidates: smallest upper end (Hi: start i1, value v1, tag n1 of OPTa[j+1] if it
      // wins) and the two smallest lower ends (L1 at start iL, L2); Ve/ie: the exact candidates;
      // gv/gi/gt: the best zero-residual start on an inexact OPTa of the group's base (its
      // interval enters the trackers at the end of the column)
      double Ve = inf, Hi = inf, L1 = inf, L2 = inf, v1 = inf, gv = inf;
      // U = min(Hi, Ve, gh), kept as each of them changes (each only decreases): the column's
      // current upper bound without recomputing it per start
      double U = inf;
      int ie = 0, i1 = 0, iL = -1, n1 = -1, gi = -1, gt = 0;
      uint64_t cand = 0;  // resolve stage: the >= 3-point starts an exact decision prices
      // (the bounds Hi, L1, L2 are only compared: v_min_f64 instead of a select pair; the values
      // that become OPTa, v1 and Ve, are selected)
      auto track = [&](int i, double v, double hi, double lo, int nt) __attribute__((always_inline)) {
        if (hi <= Hi) {
          i1 = i;
          v1 = v;
          n1 = nt;
        }
        Hi = __builtin_fmin(hi, Hi);
        U = __builtin_fmin(U, hi);
        const bool bl = lo <= L1;
        L2 = bl ? L1 : __builtin_fmin(lo, L2);
        L1 = __builtin_fmin(lo, L1);
        iL = bl ? i : iL;
      };
      // a zero-residual start (worth fl(c + OPTa[i]) in the reference) on OPTa[i] of tag tg
      // (tg < 0: inexact, tag unknown) after the pair below, in decreasing start order: rare
      // (exactly collinear segments of >= 3 points), so kept general
      double gh = inf;  // the group's upper end (early exit)
      auto zero_start = [&](int i, double v, int tg) __attribute__((always_inline)) {
        if (tg >= 0 && tg < 256) {  // exact
          if (v <= Ve) {
            Ve = v;
            ie = i;
          }
          U = __builtin_fmin(U, v);
          return;
        }
        const double w = __builtin_fma(0x1p-50, __builtin_fabs(v), Emax);
        const int ord = (!zok || tg < 0) ? 0 : gi < 0 ? 1 : tag_order(tg, gt, v, c);
        if (ord > 0) {  // the group's new best: the smaller start, value <= the old best
          gi = i;
          gt = tg;
          gv = v;
          gh = v + w;
          U = __builtin_fmin(U, gh);
        } else if (ord == 0) {
          track(i, v, v + w, v - w, tg < 0 ? -1 : tg + 1);
        }  // ord < 0: strictly above the group's best, never the first minimum
      };
      // the 1- and 2-point starts j and j-1 (residual exactly 0), select-based: the exact ones
      // give Ve/ie (the smaller start wins ties); of the inexact ones the tag order keeps one in
      // the group, and only two inexact starts of different bases leave one for the trackers
      {
        const bool has1 = j >= 1;  // wave-uniform
        const double v0 = c + opt_j, v1s = c + opt_jm1;
        const bool x0 = tg_j < 256, x1 = has1 && tg_jm1 < 256;
        const bool g0 = !x0, g1 = has1 && !x1;
        Ve = x0 ? v0 : inf;
        ie = j;
        if (x1 && v1s <= Ve) {
          Ve = v1s;
          ie = j - 1;
        }
        const int ord = (zok && g0 && g1) ? tag_order(tg_jm1, tg_j, v1s, c) : 0;
        const bool pick1 = g1 && (!g0 || ord > 0);
        gi = pick1 ? j - 1 : (g0 ? j : -1);
        gt = pick1 ? tg_jm1 : tg_j;
        gv = pick1 ? v1s : (g0 ? v0 : inf);
        gh = gv + __builtin_fma(0x1p-50, __builtin_fabs(gv), Emax);
        const bool left = g0 && g1 && ord == 0;  // start j-1 beside the group's start j
        if (__ballot(left)) {
          if (left) {
            const double w = __builtin_fma(0x1p-50, __builtin_fabs(v1s), Emax);
            track(j - 1, v1s, v1s + w, v1s - w, tg_jm1 + 1);
          }
        }
      }
      U = __builtin_fmin(__builtin_fmin(Hi, Ve), gh);
      // prefix bound for the early exit below: every segment ending at j has Syy <= SyyAll
      wx0 = L.xn[j][lane];
      wy0 = (double)L.ys[j][lane];
      SyyAll = __builtin_fma(wy0, wy0, SyyAll);
      auto add_xy = [&](int xi, double yi) {
        Sx += xi;
        Sxx += xi * xi;
        Sy += yi;
        Sxy = __builtin_fma((double)xi, yi, Sxy);
        Syy = __builtin_fma(yi, yi, Syy);
      };
      // the early-exit bound's screening slack, the same for every start of the column
      const double slack = 4.0 * kScreen * SyyAll * (1.0 + 0x1p-49);
      // start i (>= 3 points) priced from the current sums: value v, its interval [lo, hi] around
      // the reference value (tg: tag of OPTa[i]), the early-exit bound for the starts below, and
      // whether the segment is exactly collinear with a residual that rounds away (zr)
      // returns whether the interval reaches a zero residual (zero_test decides, where it can
      // matter)
      auto price = [&](int i, double o, int tg, double& v, double& hi, double& lo,
                       double& bnd) __attribute__((always_inline)) {
        // closed-form SSE: (m*Syy - Sy^2 - N1^2/D) / m, one reciprocal
        const int m = j - i + 1;  // wave-uniform, >= 3
        const double md = (double)m;
        const double D = (double)dmul24(m, Sxx, Sx);
        const double t1 = __builtin_fma(md, Syy, -(Sy * Sy));
        const double N1 = __builtin_fma(md, Sxy, -((double)Sx * Sy));
        const double den = md * D;
        double r = __builtin_amdgcn_rcp(den);
        r = __builtin_fma(r, __builtin_fma(-den, r, 1.0), r);
        const double e = __builtin_fmax(__builtin_fma(t1, D, -(N1 * N1)) * r, 0.0);
        v = (e + c) + o;  // o = OPTa[i]
        // interval around the reference value: OPT bound + screening bound of this segment +
        // the rounding of this candidate's own two additions
        const double wopt = (tg >= 0 && tg < 256) ? 0.0 : Emax;
        const double ws = kScreen * Syy;
        const double w = __builtin_fma(0x1p-50, __builtin_fabs(v), ws + wopt);
        hi = v + w;
        lo = v - w;
        bnd = dp_start_bound_slack(e, o, wopt, c, slack);
        return e <= ws;  // (zlane applied by the caller: see zmask)
      };
      // exactly collinear with a residual that rounds away (lt_pixel.h kZero, sse_exact_zero), on
      // sums of integer data (exact binary64 integers)
      auto zero_test = [&](int m, int sx, int sxx, double sy, double sxy, double syy)
                           __attribute__((always_inline)) {
        const double md = (double)m;
        const double D = (double)dmul24(m, sxx, sx);
        const double t1 = __builtin_fma(md, syy, -(sy * sy));
        const double N1 = __builtin_fma(md, sxy, -((double)sx * sy));
        // (wx0: the year offset of point j, the segment's largest)
        return zero_bound(wx0) * syy < 0x1p-54 * c && sse_exact_zero(t1, D, N1);
      };
      // a start of >= 3 points: a zero-residual start (v recomputed as the reference's
      // fl(c + OPTa[i])) or an interval candidate that starts a new base if it wins
      auto offer = [&](int i, double o, int tg, double v, double hi, double lo, bool zr) __attribute__((always_inline)) {
        if (zr) {
          zero_start(i, c + o, tg);
          hi = inf;  // kept out of the trackers (an infinite upper end never decides)
          lo = inf;
        }
        track(i, v, hi, lo, -1);
      };
      // the 1- and 2-point starts (priced above) only add their points to the sums
      add_xy(wx0, wy0);
      if (j >= 1) add_xy(wx1, wy1);
      // an upper bound on the column minimum so far (it only decreases as starts are added). A
      // start whose lower end lies above it can change no decision: it is neither the smallest
      // upper end nor among the lower ends at or below the final minimum bound H
      auto upper = [&]() __attribute__((always_inline)) { return U; };
      // start i (>= 3 points, its point already in the sums): priced, offered to the trackers when
      // its lower end reaches the column's current upper bound (else it can change no decision),
      // its early-exit bound returned
      auto one_start = [&](int i, double o, int tg) __attribute__((always_inline)) {
        double v, hi, lo, bnd;
        const bool nz = price(i, o, tg, v, hi, lo, bnd);
        // resolve stage: every start whose interval reaches the column's current upper bound (a
        // NaN bound included) is a candidate of an exact decision
        if constexpr (EXACT) {
          if (!(lo > upper())) cand |= 1ull << i;
        }
        // (each ballot of a single compare, masked by a ballot taken once: a ballot of a compound
        // condition is materialised in a VGPR as 0 / 1 and compared again, two VALU per test)
        if (__ballot(lo <= upper())) {
          if (__ballot(nz) & zmask) {  // rare: exactly collinear candidates
            const bool zr = zlane && nz && zero_test(j - i + 1, Sx, Sxx, Sy, Sxy, Syy);
            if (__ballot(zr)) {
              offer(i, o, tg, v, hi, lo, zr);
              return bnd;
            }
          }
          track(i, v, hi, lo, -1);
        }
        return bnd;
      };
      // early exit (dp_start_bound): once no start below i can reach an upper bound on the column
      // minimum in any lane, the column is complete; a start priced past that point lies above the
      // bound, so tracking it changes no decision. The starts go one at a time, each with its own
      // exit test (pricing two per exit test: 2115 vs 2231 Mpx/s on c2, profiles/r02_ab_dp)
      auto leave = [&](double bnd) __attribute__((always_inline)) {
        return prune && (__ballot(!(bnd > upper())) & colmask) == 0;
      };
      bool more = j >= 2;  // wave-uniform
      if (more) {  // starts j-2 and j-3 from the register window
        add_xy(wx2, wy2);
        more = !leave(one_start(j - 2, opt_jm2, tg_jm2));
        if (j >= 3 && more) {
          add_xy(wx3, wy3);
          more = !leave(one_start(j - 3, opt_jm3, tg_jm3));
        }
        more = more && j >= 3;
      }
      if (more) {  // the rest from LDS / private memory
        // the start index in an SGPR through the loop (a VGPR counter cost a VALU decrement and
        // a readfirstlane per start)
        for (int i = __builtin_amdgcn_readfirstlane(j - 4); i >= 0;
             i = __builtin_amdgcn_readfirstlane(i - 1)) {
          add_xy(L.xn[i][lane], (double)L.ys[i][lane]);
          // tags are kept in the window only: a start from private memory is exact or not
          if (leave(one_start(i, OPTa[i], ((exact >> i) & 1) ? 0 : -1))) break;
        }
      }
      // the group's best enters the trackers (an empty group: gv = inf, no effect)
      {
        const double w = __builtin_fma(0x1p-50, __builtin_fabs(gv), Emax);
        track(gi, gv, gv + w, gv - w, gt + 1);
      }
      const double H = __builtin_fmin(Hi, Ve);  // the exact minimum lies in [min(L1, Ve), H]
      int a, tnew;
      double vnew, enew = 0.0;
      bool xres = false;  // resolve stage: this lane decides the column exactly
      if (L1 > H) {  // no inexact interval reaches H: the exact candidates decide
        a = ie;
        vnew = Ve;
        tnew = 0;
      } else if (iL == i1 && L2 > H && Ve > H) {  // one candidate lies below all others
        a = i1;
        vnew = v1;
        // a zero-residual winner adds c to its OPTa's tag; any other starts a new base
        tnew = n1 >= 0 ? n1 : (j + 1) << 8;
        // its half-width, rounded up: Hi = fl(v1 + w1) >= v1 + w1 - ulp(Hi) / 2
        enew = __builtin_fma(Hi - v1, 1.0 + 0x1p-50, 0x1p-50 * __builtin_fabs(Hi));
      } else {
        if constexpr (EXACT) xres = col;
        else if (col) amb |= 1ull << j;
        a = v1 <= Ve ? i1 : ie;
        vnew = v1 <= Ve ? v1 : Ve;
        tnew = (j + 1) << 8;
        const double Lo = __builtin_fmin(L1, Ve);
        enew = (H - Lo) * (1.0 + 0x1p-40) + 0x1p-50 * __builtin_fabs(vnew);
      }
      if constexpr (EXACT) {
        // resolve stage: an ambiguous column is decided exactly here, so no interval widens
        // Emax and the next columns keep their certified decisions. The candidates are the
        // starts whose interval reaches H; each is worth fl(fl(e + c) + OPT[i]) with e the
        // emulated LAPACK residual (0 for 1-2 points) and OPT[i] the reference value: where OPTa[i]
        // is not exact yet, the links of its optimal prefix (argmins of decided columns, each
        // the reference's) are priced first, in increasing order, each made exact once.
        if (__ballot(xres)) resolve_column(j, xres, H, cand, opt_j, tg_j, opt_jm1, tg_jm1, a, vnew);
        if (xres) {
          tnew = 0;
          enew = 0.0;
        }
      }
      if (col) {
        ag_set(j, a);
        OPTa[j + 1] = vnew;  // wave-uniform index
        if (tnew < 256) exact |= 2ull << j;
        Emax = __builtin_fmax(enew, Emax);
        opt_jm3 = vnew;  // OPTa[j+1]: the slot of OPTa[j-3], which no later column reads
        tg_jm3 = tnew;
      }
    };
    if constexpr (EXACT) {
      // resolve stage: one column per iteration (its exact decisions are code the unrolled loop
      // below would hold four times), the window rotated by register moves
      for (int jj = 0; jj < nmax; jj++) {
        const int j = __builtin_amdgcn_readfirstlane(jj);
        column(j, xA, xB, xC, xD, yA, yB, yC, yD, oA, oB, oC, oD, gA, gB, gC, gD);
        const int xt = xD;
        xD = xC;
        xC = xB;
        xB = xA;
        xA = xt;
        const double yt = yD;
        yD = yC;
        yC = yB;
        yB = yA;
        yA = yt;
        const double ot = oD;
        oD = oC;
        oC = oB;
        oB = oA;
        oA = ot;
        const int gt = gD;
        gD = gC;
        gC = gB;
        gB = gA;
        gA = gt;
      }
    } else
    for (int jj = 0; jj < nmax; jj += 4) {
      const int j = __builtin_amdgcn_readfirstlane(jj);  // column index in an SGPR
      column(j, xA, xB, xC, xD, yA, yB, yC, yD, oA, oB, oC, oD, gA, gB, gC, gD);
      if (j + 1 < nmax)
        column(j + 1, xD, xA, xB, xC, yD, yA, yB, yC, oD, oA, oB, oC, gD, gA, gB, gC);
      if (j + 2 < nmax)
        column(j + 2, xC, xD, xA, xB, yC, yD, yA, yB, oC, oD, oA, oB, gC, gD, gA, gB);
      if (j + 3 < nmax)
        column(j + 3, xB, xC, xD, xA, yB, yC, yD, yA, oB, oC, oD, oA, gB, gC, gD, gA);
    }
    // find_segments (utils.py:633-644): starts of the optimal segments + the last point
    if (n >= 1) {
      vmask = 1ull << (n - 1);
      for (int j = n - 1; j >= 0;) {
        const int a = ag_get(j);
        if ((amb >> j) & 1) deferred = true;
        vmask |= 1ull << a;
        j = a - 1;
      }
    }
  }
  probe.mark(2);
  if constexpr (Probe::kStopAfter == 2) return kDone;
  // deferred lanes stay in the wave (the loops below use wave collectives) but do nothing more
  if (deferred) vmask = 0;

  // ---- vertices2eqns + eqns2fitted_points (utils.py:646-722) ----
  // per-year planes requested (launch-uniform)
#ifdef LT_SPEC_YEAR_OUT
  constexpr bool year_out = LT_SPEC_YEAR_OUT != 0;
#else
  const bool year_out = out.val_fit || out.fit_m || out.fit_b || out.right_m || out.right_b ||
                        out.spike || out.vertex;
#endif
  RuleState1 rs[RMAX];
  double prev_fit = 0.0;
  int32_t prev_year = 0;
  // parse_disturbances / match_rule (classes.py:156-232): the segment ending at vertex q > 0
  auto offer_rules = [&](int q, int32_t yr, double fit_vertex) __attribute__((always_inline)) {
    if (q > 0) {
#pragma unroll
      for (int r = 0; r < RMAX; r++)
        if (r < LT_NRULES)
          rs[r].offer(LT_RULE(r), LT_PRE_MODE, prev_year, yr - prev_year, prev_fit,
                      prev_fit - fit_vertex, status);
    }
    prev_fit = fit_vertex;
    prev_year = yr;
  };
  // the compact trendline (launch-uniform; lt_abi.hip trendline_expand_kernel writes the per-year
  // planes from it)
#ifdef LT_SPEC_TL_SPLIT
  constexpr bool tl_split = LT_SPEC_TL_SPLIT != 0;
#else
  const bool tl_split = tl_bits != nullptr;
#endif
  if (year_out && tl_split) {
    // ---- compact trendline: the per-year planes are NOT written here. Lockstep over the vertex
    // number q: one LAPACK-emulated fit per segment (vertices2eqns, utils.py:646-669), the
    // fitted value at each vertex (eqns2fitted_points, utils.py:682-722: the closer of the left
    // and the right eqn to the raw value, the left on a tie) for the rule offers, and per pixel
    //   tl_eqn[q][p] = (m, b) of segment q (vertex q to vertex q+1), q < n_vertices - 1,
    //   tl_bits[0][p] = present year slots (0: the reference raises for the pixel),
    //   tl_bits[1][p] = spike flags by present index, tl_bits[2][p] = vertices by non-spike
    //   index, tl_bits[3][p] = vertex q took the left eqn for its fitted value.
    // trendline_expand_kernel then writes every year row from these, one thread per (pixel,
    // year) with no store-then-load order inside a thread: here no year row is stored before a
    // fit's x-set table loads (a load after stores waits for all of them on gfx950's one
    // vector-memory counter: the year-major loop below spent ~2.7 ms of a 12.4 ms c5 launch
    // there). The eqn of segment q is stored after segment q+1's table loads are
    // issued, so those loads do not wait for it.
    const bool emit = live && !deferred;
    const bool good = emit && ok;
    const uint64_t vm = good ? vmask : 0;
    const int nv = __builtin_popcountll(vm);
    const int nvmax = wave_max(nv);
    uint64_t vrem = vm, left = 0;
    double pm = 0.0, pb = 0.0;  // eqn of vertex q-1
    double* const eq = tl_eqn;
    const int64_t np = in.n_pix;
    for (int q = 0; q < nvmax; q++) {
      const bool act = q < nv;
      const int ka = act ? __builtin_ctzll(vrem) : 0;
      if (act) vrem &= vrem - 1;
      const bool has_next = act && q + 1 < nv;
      const int kb = has_next ? __builtin_ctzll(vrem) : ka;
      double cm = pm, cb = pb;
      if (__ballot(has_next)) {
        double sm = 0.0, sbv = 0.0;
        const int rc = lsq_fit_lockstep(
            has_next, has_next ? kb - ka + 1 : 2,
            [&](int k) { return (int)L.xn[(has_next ? ka : 0) + k][lane]; },
            [&](int k) { return (double)L.ys[(has_next ? ka : 0) + k][lane]; }, xtab, sm, sbv);
        if (has_next) {
          if (rc < 0) status |= LT_ST_NUMERIC;
          cm = sm;
          cb = sbv;
          // one 16-byte store per lane, rows [q][p] coalesced across the wave
          typedef double d2 __attribute__((ext_vector_type(2)));
          d2 v;
          v.x = cm;
          v.y = cb;
          __builtin_nontemporal_store(v, (d2*)(eq + 2 * ((int64_t)q * np + p)));
        }
      }
      const double raw_v = act ? (double)L.ys[ka][lane] : 0.0;
      const double x = act ? (double)L.xn[ka][lane] : 0.0;  // the vertex's year offset
      double fit_vertex = (cm * x) + cb;
      if (q > 0 && !(pm == cm && pb == cb)) {
        const double fl = (pm * x) + pb;
        if (__builtin_fabs(fl - raw_v) <= __builtin_fabs(fit_vertex - raw_v)) {
          fit_vertex = fl;
          left |= 1ull << q;
        }
      }
      if (act) offer_rules(q, y0 + L.xn[ka][lane], fit_vertex);
      pm = cm;
      pb = cb;
    }
    if (emit) {
      __builtin_nontemporal_store(good ? pres : 0ull, tl_bits + p);
      __builtin_nontemporal_store(spike, tl_bits + np + p);
      __builtin_nontemporal_store(vm, tl_bits + 2 * np + p);
      __builtin_nontemporal_store(left, tl_bits + 3 * np + p);
    }
  } else if (year_out) {
    // Year-major: every year slot is one wave-uniform step and each per-year plane is written
    // one coalesced row at a time (lane l -> pixel p, all lanes the same year). A lane reaching
    // a vertex that has a next vertex needs that segment's fit (lanes without a next vertex reuse
    // the previous equation, utils.py:662). The fits are LAPACK-emulated in lockstep, and each
    // lane keeps one fit ahead: a fit step is issued only in a year where some lane reaches such
    // a vertex with its lookahead slot empty, and in it every lane whose slot is free (or is being
    // used this year) fits its next segment. A wave then issues about as many fit steps as its
    // lanes have vertices (the lower bound), not one per year. Deferred and dead lanes write
    // nothing (the resolve stage writes them).
    const bool emit = live && !deferred;
    const bool good = emit && ok;
    uint64_t vrem = vmask;           // vertices not reached yet (non-spike indices)
    uint64_t frem = vmask;           // vertices whose segment is not fitted yet (the lowest next)
    double pm = 0.0, pb = 0.0;       // eqn of the previous vertex
    double cm = 0.0, cb = 0.0;       // eqn of the current vertex (right eqn of the points)
    double nm = 0.0, nb = 0.0;       // lookahead: eqn of the segment from the next vertex
    bool have_n = false;
    // spike / vertex flags by year slot: with yflags the u8 planes are written from them by
    // year_flags_kernel (lt_abi.hip) in 256-byte rows instead of 64-byte pieces here
    uint64_t spk = 0, vtx = 0;
    int t = 0, k = 0, q = 0;         // present index, non-spike index, vertex number
    // One year's row of the five binary64 planes. (A fit step's x-set table loads share the
    // in-order vector-memory counter with the stores, so a load issued after a year's stores waits
    // for all of them (s_waitcnt vmcnt(0)); holding each row a year or two and storing it after
    // the next fit step spilled the held rows: c5 1060 / 928 vs 1260 Mpx/s, profiles/r04_run16.)
    struct Row {
      double fv, fm, fb, rm, rb;
      bool pr;  // the year is present in this lane
      bool uni;  // ... in every emitting lane (no NaN selects)
    };
    // (16-byte stores of pixel pairs from the even lanes, the odd lane's value moved over by DPP:
    // c5 1083-1092 vs 1260 Mpx/s, profiles/r04_run19)
    auto store_row = [&](int yy, const Row& r) __attribute__((always_inline)) {
      const int64_t o = LT_AB_YEAR_SINK ? p : (int64_t)yy * os + p;
      // write-once planes: nontemporal stores (same-box c5 A/B: 1012 vs 896-925 Mpx/s). When
      // the year is present in every emitting lane (always, without a cloud mask) the values
      // are stored as they are: no NaN select pair per plane
      auto put = [&](double* plane, double v) __attribute__((always_inline)) {
        if (plane && !LT_AB_NO_YEAR_STORES) {
          if (LT_AB_YEAR_SINK == 2 || !LT_YEAR_NT)
            plane[o] = v;
          else
            year_row_store(v, plane + o);
        }
      };
      if (r.uni) {
        put(LT_OUTF(out, val_fit), r.fv);
        put(LT_OUTF(out, fit_m), r.fm);
        put(LT_OUTF(out, fit_b), r.fb);
        put(LT_OUTF(out, right_m), r.rm);
        put(LT_OUTF(out, right_b), r.rb);
      } else {
        put(LT_OUTF(out, val_fit), r.pr ? r.fv : nan);
        put(LT_OUTF(out, fit_m), r.pr ? r.fm : nan);
        put(LT_OUTF(out, fit_b), r.pr ? r.fb : nan);
        put(LT_OUTF(out, right_m), r.pr ? r.rm : nan);
        put(LT_OUTF(out, right_b), r.pr ? r.rb : nan);
      }
    };
    for (int y = 0; y < Y; y++) {    // wave-uniform
      const bool pr = good && ((pres >> y) & 1);
      const bool sp = pr && ((spike >> t) & 1);
      const bool isv = pr && !sp && ((vrem >> k) & 1);
      const uint64_t after = vrem & (vrem - 1);  // vertices after this one
      const bool nextfit = isv && after != 0;
      double sm = 0.0, sbv = 0.0;
      bool fitnow = false;
      if (__ballot(nextfit && !have_n) && !LT_AB_NO_FITS) {
        const uint64_t fnext = frem & (frem - 1);
        fitnow = fnext != 0 && (!have_n || nextfit);
        const int kbase = fitnow ? __builtin_ctzll(frem) : 0;
        const int kb = fitnow ? __builtin_ctzll(fnext) : 1;
        const int rc = lsq_fit_lockstep(
            fitnow, kb - kbase + 1, [&](int i) { return (int)L.xn[kbase + i][lane]; },
            [&](int i) { return (double)L.ys[kbase + i][lane]; }, xtab, sm, sbv);
        if (fitnow) {
          if (rc < 0) status |= LT_ST_NUMERIC;
          frem = fnext;
        }
      }
      if (nextfit) {
        pm = cm;
        pb = cb;
        cm = have_n ? nm : sm;
        cb = have_n ? nb : sbv;
        have_n = have_n && fitnow;  // the slot was used: refilled by this year's step
      } else {
        have_n = have_n || fitnow;
      }
      if (have_n && fitnow) {
        nm = sm;
        nb = sbv;
      }

      if (isv && !nextfit) {  // the last vertex: left eqn = right eqn = the previous one
        pm = cm;
        pb = cb;
      }
      const double x = (double)(L.year[y] - y0);
      double fv = (cm * x) + cb, fmv = cm, fbv = cb;
      if (isv && q > 0 && !(pm == cm && pb == cb)) {
        const double raw_v = (double)L.ys[k][lane];
        const double fl = (pm * x) + pb;
        if (__builtin_fabs(fl - raw_v) <= __builtin_fabs(fv - raw_v)) {
          fv = fl;
          fmv = pm;
          fbv = pb;
        }
      }
      if (isv) {
        offer_rules(q, L.year[y], fv);
        vrem = after;
        q++;
      }
      {  // absent years and pixels the reference raises for: NaN / 0
        const Row row{fv, fmv, fbv, cm, cb, pr, __ballot(emit && !pr) == 0};
        if (emit) store_row(y, row);
      }
      if (emit) {
        const int64_t o = (int64_t)y * os + p;
        if (yflags) {
          spk |= (uint64_t)sp << y;
          vtx |= (uint64_t)isv << y;
        } else {
          if (auto* a = LT_OUTF(out, spike)) a[o] = sp ? 1 : 0;
          if (auto* a = LT_OUTF(out, vertex)) a[o] = isv ? 1 : 0;
        }
      }
      if (pr) {
        if (!sp) k++;
        t++;
      }
    }
    if (emit && yflags) {
      yflags[p] = spk;
      yflags[in.n_pix + p] = vtx;
    }
  } else if constexpr (RMAX <= LT_CERT_RULES) {
    // (the resolve stage too: c2 2387 vs 2376 Mpx/s, resolve 0.43 vs 0.46 ms, profiles/r04_run8)
    // ---- labels only, certified. The rules need the fitted values at the vertices, and only the
    // winners' values bit-exactly. (A) lockstep over the vertex number q: each segment's fit by
    // the closed form, the fitted value at each vertex as an interval around the reference's
    // (kFitW), and each disturbance offered to the rules' candidate sets (lt_pixel.h RuleCands);
    // (B) lockstep over the candidates: the emulated (reference) fits of the two or three
    // segments around each, and the exact offers, in order, to the rules holding it ----
    const int nv = __builtin_popcountll(vmask);
    const int nvmax = wave_max(nv);
    RuleCands cand[RMAX];
    uint64_t vrem = vmask;  // vertices from q on: vertex q is its lowest bit
    // closed-form eqn (slope, intercept, error scale) of the segment ending at vertex q-1
    double am = 0.0, ab = 0.0, asc = 0.0;
    double fprev = 0.0, wprev = 0.0;  // fitted value of vertex q-1: center, half-width
    int32_t yprev = 0;
    // interior vertices (by point index) whose fitted value certainly takes the left (CL) / the
    // right (CR) eqn: the reference's choice, decided by the closed-form intervals (pass B then
    // needs only that eqn's emulated fit there)
    uint64_t CL = 0, CR = 0;
    auto add_pt = [&](int k, int& Sx, int& Sxx, double& Sy, double& Sxy, double& ymx)
                      __attribute__((always_inline)) {
      const int xi = L.xn[k][lane];
      const double yi = (double)L.ys[k][lane];
      Sx += xi;
      Sxx += xi * xi;
      Sy += yi;
      Sxy = __builtin_fma((double)xi, yi, Sxy);
      ymx = __builtin_fmax(ymx, __builtin_fabs(yi));
    };
    for (int q = 0; q < nvmax; q++) {
      const bool act = q < nv;
      const int ka = act ? __builtin_ctzll(vrem) : 0;
      if (act) vrem &= vrem - 1;
      const bool has_next = act && q + 1 < nv;
      const int kb = has_next ? __builtin_ctzll(vrem) : ka;
      double cm = am, cb = ab, csc = asc;  // the last vertex reuses the previous eqn (utils.py:662)
      if (__ballot(has_next)) {
        // least squares of the points ka..kb by the closed form: two to four points straight-line,
        // longer segments in a loop the wave takes only if some lane has one
        const int m = kb - ka + 1;
        int Sx = 0, Sxx = 0;
        double Sy = 0.0, Sxy = 0.0, ymx = 0.0;
        if (has_next) {
          add_pt(ka, Sx, Sxx, Sy, Sxy, ymx);
          add_pt(ka + 1, Sx, Sxx, Sy, Sxy, ymx);
          if (m >= 3) add_pt(ka + 2, Sx, Sxx, Sy, Sxy, ymx);
          if (m >= 4) add_pt(ka + 3, Sx, Sxx, Sy, Sxy, ymx);
        }
        const bool longer = has_next && m > 4;
        if (__ballot(longer)) {
          const int mmax = wave_max(longer ? m : 0);
          for (int k = 4; k < mmax; k++)
            if (k < m) add_pt(ka + k, Sx, Sxx, Sy, Sxy, ymx);
        }
        if (has_next) {
          const double md = (double)m;
          const double D = (double)(m * Sxx - Sx * Sx);  // > 0: distinct x
          const double N1 = __builtin_fma(md, Sxy, -((double)Sx * Sy));
          double r = __builtin_amdgcn_rcp(D);
          r = __builtin_fma(r, __builtin_fma(-D, r, 1.0), r);
          double rm = __builtin_amdgcn_rcp(md);
          rm = __builtin_fma(rm, __builtin_fma(-md, rm, 1.0), rm);
          cm = N1 * r;
          cb = __builtin_fma(-cm, (double)Sx, Sy) * rm;
          csc = __builtin_fma(__builtin_fabs(cm), 64.0, __builtin_fabs(cb)) + ymx;
          // a segment reaching past year offset 63: kFitWide (lt_pixel.h fit_width)
          csc *= fit_width_factor(L.xn[kb][lane]);
        }
      }
      // the fitted value at vertex q (eqns2fitted_points: the closer of the left and right eqn)
      const double x = act ? (double)L.xn[ka][lane] : 0.0;
      const double raw_v = act ? (double)L.ys[ka][lane] : 0.0;
      const double fr = (cm * x) + cb, wr = kFitW * csc;
      double fv = fr, w = wr;
      if (q > 0 && has_next) {
        const double fl = (am * x) + ab, wl = kFitW * asc;
        const double dl = __builtin_fabs(fl - raw_v), dr = __builtin_fabs(fr - raw_v);
        const double slack = wl + wr + 0x1p-50 * (dl + dr);
        if (dl + slack <= dr) {  // certainly the left eqn
          fv = fl;
          w = wl;
          CL |= 1ull << ka;
        } else if (!(dr + slack < dl)) {  // either: the hull of both intervals
          const double lo = __builtin_fmin(fl - wl, fr - wr), hi = __builtin_fmax(fl + wl, fr + wr);
          fv = 0.5 * (lo + hi);
          w = 0.5 * (hi - lo) + 0x1p-50 * (__builtin_fabs(lo) + __builtin_fabs(hi));
        } else {  // certainly the right eqn
          CR |= 1ull << ka;
        }
      }
      const int32_t yr = y0 + (int32_t)x;
      if (act && q > 0) {  // the disturbance from vertex q-1 to vertex q (classes.py:156-176)
        const double mag = fprev - fv;
        const double wm = (wprev + w) + 0x1p-50 * (__builtin_fabs(fprev) + __builtin_fabs(fv));
#pragma unroll
        for (int r = 0; r < RMAX; r++)
          if (r < LT_NRULES)
            cand[r].offer(LT_RULE(r), LT_PRE_MODE, yprev, yr - yprev, fprev - wprev,
                          fprev + wprev, mag - wm, mag + wm, 1ull << ka, status);
      }
      am = cm;
      ab = cb;
      asc = csc;
      fprev = fv;
      wprev = w;
      yprev = yr;
    }
    // (B) the candidates in increasing order; a series with an infinite value (whose emulated
    // fits fail and are flagged) replays every disturbance
    uint64_t U = 0;
#pragma unroll
    for (int r = 0; r < RMAX; r++)
      if (r < LT_NRULES) U |= cand[r].G;
    if (infdata) U = vmask & (vmask - 1);
    const int nu = __builtin_popcountll(U);
    const int numax = wave_max(nu);
    for (int it = 0; it < numax; it++) {
      const bool act = it < nu;
      const int kq = act ? __builtin_ctzll(U) : 1;  // end vertex of the disturbance (>= 1)
      if (act) U &= U - 1;
      const uint64_t below = act ? vmask & ((1ull << kq) - 1) : 1;  // the vertices before kq
      const int k1 = 63 - __builtin_clzll(below);                     // vertex q-1
      const uint64_t below2 = below & ~(1ull << k1);
      const bool has2 = act && below2 != 0;
      const int k2 = has2 ? 63 - __builtin_clzll(below2) : 0;         // vertex q-2
      const uint64_t above = act ? vmask & ~((2ull << kq) - 1) : 0;    // (kq = 63: none)
      const bool hasn = above != 0;
      const int kn = hasn ? __builtin_ctzll(above) : 0;               // vertex q+1
      // the reference's eqns (vertices2eqns, utils.py:646-669): e1 of segment q-1 (k1..kq),
      // e2 of segment q-2 (k2..k1), e3 of segment q (kq..kn)
      // the fitted value at vertex q-1 takes e2 (left) or e1 (right), at vertex q e1 (left) or
      // e3 (right): where pass A's intervals decided the side, only that eqn is fitted. A lane
      // then needs at most two of the three (the third only at an undecided vertex), fitted in
      // lockstep slots over the wave's largest count (three fixed steps: one always wasted).
      // Each eqn is kept only as its values at the two vertices (fl1 / fr1 at vertex q-1, flq /
      // frq at vertex q), all the choice needs: where two eqns are identical their values are,
      // so the reference's "same eqn: the right one" shortcut gives the same value
      // (LT_PASSB_SLOTS=0, A/B runs: the three eqns always, each fitted whenever a lane has it)
      const bool slots = ((LT_PASSB_SLOTS >> (EXACT ? 1 : 0)) & 1) && !infdata;
      const bool cl1 = slots && has2 && ((CL >> k1) & 1), cr1 = slots && has2 && ((CR >> k1) & 1);
      const bool clq = slots && hasn && ((CL >> kq) & 1), crq = slots && hasn && ((CR >> kq) & 1);
      unsigned todo = (act && !(cl1 && crq) ? 1u : 0u) | (has2 && !cr1 ? 2u : 0u) |
                      (hasn && !clq ? 4u : 0u);
      const int nfit = wave_max(__builtin_popcount(todo));
      double fl1 = 0.0, fr1 = 0.0, flq = 0.0, frq = 0.0;
#pragma unroll
      for (int sl = 0; sl < 3; sl++) {  // unrolled (a loop spilled 13-51 VGPRs across the fit)
        if (sl >= nfit) break;           // wave-uniform
        const bool on = todo != 0;
        const int which = on ? __builtin_ctz(todo) : 0;  // 0: e1, 1: e2, 2: e3
        if (on) todo &= todo - 1;
        const int k0 = which == 0 ? k1 : which == 1 ? k2 : kq;
        const int k9 = which == 0 ? kq : which == 1 ? k1 : kn;
        if (__ballot(on)) {
          double sm = 0.0, sb = 0.0;
          const int rc = lsq_fit_lockstep(
              on, k9 - k0 + 1, [&](int i) { return (int)L.xn[k0 + i][lane]; },
              [&](int i) { return (double)L.ys[k0 + i][lane]; }, xtab, sm, sb);
          if (on) {
            if (rc < 0) status |= LT_ST_NUMERIC;
            const double x1 = (double)L.xn[k1][lane], xq = (double)L.xn[kq][lane];
            if (which == 0) {
              fr1 = (sm * x1) + sb;
              flq = (sm * xq) + sb;
            } else if (which == 1) {
              fl1 = (sm * x1) + sb;
            } else {
              frq = (sm * xq) + sb;
            }
          }
        }
      }
      // fitted values at vertices q-1 and q, as the walk computes them (the closer eqn to the raw
      // value, the left on a tie; a side pass A decided directly)
      auto pick = [&](int k, bool left, bool right, double fl, double fr)
                      __attribute__((always_inline)) {
        if (left) return fl;
        if (right) return fr;
        const double raw_v = (double)L.ys[k][lane];
        return __builtin_fabs(fl - raw_v) <= __builtin_fabs(fr - raw_v) ? fl : fr;
      };
      const double f1 = has2 ? pick(k1, cl1, cr1, fl1, fr1) : fr1;
      const double fq = hasn ? pick(kq, clq, crq, flq, frq) : flq;
      const int32_t on = y0 + (int32_t)L.xn[k1][lane];
      const int32_t du = (int32_t)L.xn[kq][lane] - (int32_t)L.xn[k1][lane];
#pragma unroll
      for (int r = 0; r < RMAX; r++)
        if (r < LT_NRULES && act && (infdata || ((cand[r].G >> kq) & 1)))
          rs[r].offer(LT_RULE(r), LT_PRE_MODE, on, du, f1, f1 - fq, status);
    }
  } else {
    // labels only, in lockstep over the vertex number q: the fitted value at each vertex is all
    // the rules need
    const int nv = __builtin_popcountll(vmask);
    const int nvmax = wave_max(nv);
    uint64_t vrem = vmask;  // vertices from q on: vertex q is its lowest bit
    double pm = 0.0, pb = 0.0;   // eqn of vertex q-1
    for (int q = 0; q < nvmax; q++) {
      const bool act = q < nv;
      const int ka = act ? __builtin_ctzll(vrem) : 0;
      if (act) vrem &= vrem - 1;
      const bool has_next = act && q + 1 < nv;
      const int kb = has_next ? __builtin_ctzll(vrem) : ka;
      double cm = pm, cb = pb;
      // one LAPACK-emulated fit per vertex number for the whole wave (lanes without a next
      // vertex reuse the previous equation, utils.py:662)
      const int mseg = has_next ? kb - ka + 1 : 2;
      const int kbase = has_next ? ka : 0;
      double sm = 0.0, sbv = 0.0;
      if (__ballot(has_next)) {
        const int rc = lsq_fit_lockstep(
            has_next, mseg, [&](int k) { return (int)L.xn[kbase + k][lane]; },
            [&](int k) { return (double)L.ys[kbase + k][lane]; }, xtab, sm, sbv);
        if (has_next) {
          if (rc < 0) status |= LT_ST_NUMERIC;
          cm = sm;
          cb = sbv;
        }
      }
      const double raw_v = act ? (double)L.ys[ka][lane] : 0.0;
      const double x = act ? (double)L.xn[ka][lane] : 0.0;  // the vertex's year offset
      double fit_vertex;
      if (q > 0 && !(pm == cm && pb == cb)) {
        const double fl = (pm * x) + pb;
        const double fr = (cm * x) + cb;
        fit_vertex = __builtin_fabs(fl - raw_v) <= __builtin_fabs(fr - raw_v) ? fl : fr;
      } else {
        fit_vertex = (cm * x) + cb;
      }
      if (act) offer_rules(q, y0 + L.xn[ka][lane], fit_vertex);
      pm = cm;
      pb = cb;
    }
  }

  probe.mark(3);
  if constexpr (Probe::kStopAfter == 3) return kDone;
  // ---- change_labeling (utils.py:795-820) outputs ----
  if (live && !deferred) {
#pragma unroll
    for (int r = 0; r < RMAX; r++)
      if (r < LT_NRULES) rs[r].write(LT_RULE(r), out, (int64_t)r * os + p);
  }
  probe.mark(4);
  if (!live || deferred) {
    if (!deferred) return kDone;
    if constexpr (EXACT) {  // a binary32 resolve given a value binary32 cannot hold: unreachable
      if (auto* a = LT_OUTF(out, status)) a[p] = status | LT_ST_NUMERIC;
      return kDone;
    }
    return f32_bad ? kDeferWide : kDeferExact;
  }
  if (auto* a = LT_OUTF(out, n_years)) a[p] = T;
  if (auto* a = LT_OUTF(out, status)) a[p] = status;
  return kDone;
}

}  // namespace lt
