// lt_pixel.h — the per-pixel LandTrendr pipeline as device code (one pixel per lane).
//
// Stages, in reference order (/root/reference/utils.py):
//   pick_winners :491-521   winner per calendar year (scene metadata in scalar memory)
//   despike      :556-582   numpy-pairwise std + 3-window scan over the ORIGINAL series
//   timeseries2int_series :534-554, dropna :608
//   segmented_least_squares :600-631 + find_segments :633-644   (DP, first-minimum argmin)
//   vertices2eqns :646-669, eqns2fitted_points :682-722
//   Trendline.parse_disturbances / match_rule (classes.py:156-232), change_labeling :795-820
// All arithmetic that can decide a tie is the emulated LAPACK of lt_lapack.h.
#pragma once
#ifndef __HIPCC_RTC__  // hiprtc (the JIT kernels, lt_jit.h) brings its own
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "../../include/lt_abi.h"
#include "lt_lapack.h"

// The output planes of lt_tile_out as bits (lt_jit.h out_field_mask). A JIT kernel specialised
// for a launch's output fields (LT_SPEC_FIELDS) sees every plane the launch does not write as a
// compile-time null (LT_OUTF): its code, and the values only it needs (RuleState1::init for an
// unrequested initial_val), are dropped, which frees registers in the rule-heavy instances.
#define LT_FIELD_status (1u << 0)
#define LT_FIELD_n_years (1u << 1)
#define LT_FIELD_matched (1u << 2)
#define LT_FIELD_class_val (1u << 3)
#define LT_FIELD_onset_year (1u << 4)
#define LT_FIELD_duration (1u << 5)
#define LT_FIELD_magnitude (1u << 6)
#define LT_FIELD_initial_val (1u << 7)
#define LT_FIELD_winner (1u << 8)
#define LT_FIELD_val_raw (1u << 9)
#define LT_FIELD_val_fit (1u << 10)
#define LT_FIELD_fit_m (1u << 11)
#define LT_FIELD_fit_b (1u << 12)
#define LT_FIELD_right_m (1u << 13)
#define LT_FIELD_right_b (1u << 14)
#define LT_FIELD_spike (1u << 15)
#define LT_FIELD_vertex (1u << 16)
#ifdef LT_SPEC_FIELDS
#define LT_OUTF(o, f) ((LT_SPEC_FIELDS & LT_FIELD_##f) ? (o).f : (decltype((o).f)) nullptr)
#else
#define LT_OUTF(o, f) ((o).f)
#endif

namespace lt {

// Scene metadata in device memory (uploaded once per distinct scene by lt_analyze_tile).
struct DevScene {
  int32_t n_obs;
  int32_t n_years;
  // bit y: the target is Feb-29 and year y is not a leap year (one word: a scalar load, where a
  // byte array needs a vector load — and on CDNA a vector load waits for every pending store)
  uint64_t feb29_mask;
  int32_t year[LT_MAX_YEARS];
  int32_t slot_begin[LT_MAX_YEARS + 1];
  int32_t order[LT_MAX_OBS];
  int32_t dist[LT_MAX_OBS];
  // pick_winners' winner per year slot when every observation is valid (no cloud mask): the same
  // for all pixels, so computed once per scene on the host (-1: no observation in the year)
  int32_t winner_all[LT_MAX_YEARS];
};

// numpy pairwise sum (n <= 128) of a[0..n-1]: 8 accumulators, then sequential remainder.
template <class G>
__host__ __device__ inline double np_sum(int n, G a) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; i++) r += a(i);
    return r;
  }
  double r0 = a(0), r1 = a(1), r2 = a(2), r3 = a(3), r4 = a(4), r5 = a(5), r6 = a(6), r7 = a(7);
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
    r0 += a(i); r1 += a(i + 1); r2 += a(i + 2); r3 += a(i + 3);
    r4 += a(i + 4); r5 += a(i + 5); r6 += a(i + 6); r7 += a(i + 7);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; i++) res += a(i);
  return res;
}

// change_labeling state of ONE rule: match_rule's filters (classes.py:190-211) and the FD/GD/LD
// winner replacement on strict inequality (classes.py:217-230).
struct RuleState1 {
  bool have = false;
  int32_t on = LT_NODATA, du = LT_NODATA;
  double mag = (double)LT_NODATA, init = (double)LT_NODATA;

  __host__ __device__ __attribute__((always_inline)) void offer(const lt_rule& R, int pre_mode, int32_t d_on, int32_t d_du,
                                 double d_init, double d_mag, int& status) {
    bool match = true;
    if (R.onset_op == LT_Q_EQ) match = match && ((double)d_on == R.onset_val);
    else if (R.onset_op == LT_Q_LE) match = match && !((double)d_on > R.onset_val);
    else if (R.onset_op == LT_Q_GE) match = match && !((double)d_on < R.onset_val);
    if (R.duration_op == LT_Q_GT) match = match && !((double)d_du <= R.duration_val);
    else if (R.duration_op == LT_Q_LT) match = match && !((double)d_du >= R.duration_val);
    if (R.pre_op != LT_Q_UNSET) {
      if (pre_mode == LT_PRE_REFERENCE) status |= LT_ST_PRE_THRESHOLD_ATTR;
      else if (R.pre_op == LT_Q_GT) match = match && !(d_init <= R.pre_val);
      else if (R.pre_op == LT_Q_LT) match = match && !(d_init >= R.pre_val);
    }
    if (!match) return;
    bool take = !have;
    if (have) {
      if (R.change_type == LT_CT_FD) take = d_on < on;
      else if (R.change_type == LT_CT_GD) take = d_mag > mag;
      else if (R.change_type == LT_CT_LD) take = d_du > du;
    }
    if (take) {
      have = true;
      on = d_on;
      du = d_du;
      mag = d_mag;
      init = d_init;
    }
  }

  __host__ __device__ __attribute__((always_inline)) void write(const lt_rule& R, const lt_tile_out& out, int64_t q) const {
    if (auto* a = LT_OUTF(out, matched)) a[q] = have ? 1 : 0;
    if (auto* a = LT_OUTF(out, class_val)) a[q] = have ? R.class_val : LT_NODATA;
    if (auto* a = LT_OUTF(out, onset_year)) a[q] = on;
    if (auto* a = LT_OUTF(out, duration)) a[q] = du;
    if (auto* a = LT_OUTF(out, magnitude)) a[q] = mag;
    if (auto* a = LT_OUTF(out, initial_val)) a[q] = init;
  }
};

// Vertex fitted values known only to within an interval (the labels-only analyze path prices
// every segment fit with the closed form first, lt_fast.h): the candidate set of ONE rule. match_rule
// (classes.py:185-230) keeps, among the matching disturbances, the first one of maximal key
// (GD: magnitude; LD: duration; FD: -onset, onsets increase along the trendline). Offered the
// disturbances in order, each with an interval [klo, khi] around its key and a match that is
// certain or only possible (a pre_threshold test the init interval straddles), G collects every
// disturbance that can still be the winner:
//   * khi <= lo (lo: the largest lower end among CERTAIN matches in G) -> an earlier certain match
//     is at least as large: never the first maximum;
//   * a certain match with klo > hi (hi: the largest upper end in G) -> larger than all of G, so
//     no member of G can win: G restarts from it;
//   * otherwise it joins G.
// The winner is always in G, so replaying the exact offers over G alone (RuleState1, in order)
// gives the reference's winner. G is a mask over the disturbance's end-vertex index.
struct RuleCands {
  uint64_t G = 0;
  double lo = -__builtin_inf(), hi = -__builtin_inf();

  __host__ __device__ __attribute__((always_inline)) void offer(
      const lt_rule& R, int pre_mode, int32_t d_on, int32_t d_du, double init_lo,
      double init_hi, double mag_lo, double mag_hi, uint64_t bit, int& status) {
    bool match = true, maybe = false;
    if (R.onset_op == LT_Q_EQ) match = match && ((double)d_on == R.onset_val);
    else if (R.onset_op == LT_Q_LE) match = match && !((double)d_on > R.onset_val);
    else if (R.onset_op == LT_Q_GE) match = match && !((double)d_on < R.onset_val);
    if (R.duration_op == LT_Q_GT) match = match && !((double)d_du <= R.duration_val);
    else if (R.duration_op == LT_Q_LT) match = match && !((double)d_du >= R.duration_val);
    if (R.pre_op != LT_Q_UNSET) {
      if (pre_mode == LT_PRE_REFERENCE) {
        status |= LT_ST_PRE_THRESHOLD_ATTR;
      } else if (R.pre_op == LT_Q_GT) {  // match iff !(init <= pre_val)
        const bool yes = init_lo > R.pre_val, no = init_hi <= R.pre_val;
        match = match && !no;
        maybe = maybe || !yes;
      } else if (R.pre_op == LT_Q_LT) {  // match iff !(init >= pre_val)
        const bool yes = init_hi < R.pre_val, no = init_lo >= R.pre_val;
        match = match && !no;
        maybe = maybe || !yes;
      }
    }
    if (!match) return;
    double klo = mag_lo, khi = mag_hi;
    if (R.change_type == LT_CT_FD) klo = khi = -(double)d_on;
    else if (R.change_type == LT_CT_LD) klo = khi = (double)d_du;
    if (khi <= lo) return;
    if (!maybe && klo > hi) {
      G = bit;
      lo = klo;
      hi = khi;
      return;
    }
    G |= bit;
    hi = __builtin_fmax(khi, hi);  // (bounds: v_max_f64, not a select pair)
    if (!maybe) lo = __builtin_fmax(klo, lo);
  }
};

// Half-width factor of a closed-form vertex fit against the reference's (emulated dgelsd) one:
// |fitted value - reference fitted value| <= kFitW * (|slope| * 64 + |intercept| + max|y|) at any
// year offset x < 64. tests/test_screening.py measures the emulated dgelsd and the kernel's closed
// form against the exact rational fit over adversarial segments and requires a 2^10 margin. The
// a-priori bound (DESIGN.md § Screening bounds, tests/test_screening_bounds.py) is 2^-35.4 of the
// scale for segments within offsets 0..63, but grows with the conditioning of [1, x] past that (a
// short segment at offsets near 255: 2^-31.4): such segments use 16 kFitW (fit_width_factor).
constexpr double kFitW = 0x1p-32;
__host__ __device__ inline double fit_width_factor(int x_max) { return x_max <= 63 ? 1.0 : 16.0; }

// change_labeling state for all rules (classes.py:213-230 winner bookkeeping).
struct RuleState {
  bool have[LT_MAX_RULES];
  int32_t on[LT_MAX_RULES], du[LT_MAX_RULES];
  double mag[LT_MAX_RULES], init[LT_MAX_RULES];

  __host__ __device__ void reset(int nr) {
    for (int r = 0; r < nr; r++) {
      have[r] = false;
      on[r] = LT_NODATA;
      du[r] = LT_NODATA;
      mag[r] = (double)LT_NODATA;
      init[r] = (double)LT_NODATA;
    }
  }

  // One Disturbance (classes.py:170-175) offered to every rule: match_rule's filters
  // (classes.py:190-211) then the FD/GD/LD replacement on strict inequality (:217-230).
  __host__ __device__ void offer(const lt_params& P, int32_t d_on, int32_t d_du, double d_init,
                        double d_mag, int& status) {
    for (int r = 0; r < P.n_rules; r++) {
      const lt_rule& R = P.rules[r];
      bool match = true;
      if (R.onset_op == LT_Q_EQ) match = match && ((double)d_on == R.onset_val);
      else if (R.onset_op == LT_Q_LE) match = match && !((double)d_on > R.onset_val);
      else if (R.onset_op == LT_Q_GE) match = match && !((double)d_on < R.onset_val);
      if (R.duration_op == LT_Q_GT) match = match && !((double)d_du <= R.duration_val);
      else if (R.duration_op == LT_Q_LT) match = match && !((double)d_du >= R.duration_val);
      if (R.pre_op != LT_Q_UNSET) {
        if (P.pre_threshold_mode == LT_PRE_REFERENCE) status |= LT_ST_PRE_THRESHOLD_ATTR;
        else if (R.pre_op == LT_Q_GT) match = match && !(d_init <= R.pre_val);
        else if (R.pre_op == LT_Q_LT) match = match && !(d_init >= R.pre_val);
      }
      if (!match) continue;
      bool take = !have[r];
      if (have[r]) {
        if (R.change_type == LT_CT_FD) take = d_on < on[r];
        else if (R.change_type == LT_CT_GD) take = d_mag > mag[r];
        else if (R.change_type == LT_CT_LD) take = d_du > du[r];
      }
      if (take) {
        have[r] = true;
        on[r] = d_on;
        du[r] = d_du;
        mag[r] = d_mag;
        init[r] = d_init;
      }
    }
  }

  __host__ __device__ void write(const lt_params& P, const lt_tile_out& out, int64_t p) const {
    const int64_t os = out.stride;
    for (int r = 0; r < P.n_rules; r++) {
      const int64_t q = (int64_t)r * os + p;
      if (out.matched) out.matched[q] = have[r] ? 1 : 0;
      if (out.class_val) out.class_val[q] = have[r] ? P.rules[r].class_val : LT_NODATA;
      if (out.onset_year) out.onset_year[q] = on[r];
      if (out.duration) out.duration[q] = du[r];
      if (out.magnitude) out.magnitude[q] = mag[r];
      if (out.initial_val) out.initial_val[q] = init[r];
    }
  }
};

// Screening bound: |LAPACK residual - closed-form residual| <= kScreen * sum(y^2) of the segment.
// tests/test_screening.py measures both against the exact rational SSE over ~1000 adversarial
// segments (int16-range, non-integer, large-offset, nearly collinear, gapped x, m <= 64): the
// emulated dgelsd stays within 2^-50 * sum(y^2), the kernel's closed form within 2^-49.5, their
// difference within 2^-49.5 (the test requires 2^-40): 2^-30 leaves a margin of at least 2^10.
constexpr double kScreen = 0x1p-30;

// The fused load stage (lt_abi.h lt_index_lin): the index value of the band values whose
// linear form is acc (modulo 2^64), as lt_index_apply would store it into out_type and the analyze
// stage read it back (float(val), utils.py:357): wrapped to the node type, then the store into
// out_type (lt_index.h codegen: saturation into an integer type, rounding into binary32).
__host__ __device__ inline int lin_type_bits(int t) {
  switch (t) {
    case LT_T_I8: case LT_T_U8: return 8;
    case LT_T_I16: case LT_T_U16: return 16;
    case LT_T_I32: case LT_T_U32: return 32;
    default: return 64;
  }
}
__host__ __device__ inline bool lin_type_signed(int t) {
  return t == LT_T_I8 || t == LT_T_I16 || t == LT_T_I32 || t == LT_T_I64;
}
__host__ __device__ inline void lin_out_range(int t, int64_t& lo, int64_t& hi) {
  const int b = lin_type_bits(t);
  if (b == 64) {  // I64 (a U64 store type does not exist)
    lo = (int64_t)(1ull << 63);
    hi = (int64_t)((1ull << 63) - 1);
  } else if (lin_type_signed(t)) {
    lo = -(int64_t)(1ull << (b - 1));
    hi = (int64_t)(1ull << (b - 1)) - 1;
  } else {
    lo = 0;
    hi = (int64_t)((1ull << b) - 1);
  }
}
__host__ __device__ inline double lin_store(const lt_index_lin& L, uint64_t acc) {
  const int bits = lin_type_bits(L.wrap_type);
  int64_t r = (int64_t)acc;
  if (bits < 64) {
    const int sh = 64 - bits;
    r = lin_type_signed(L.wrap_type) ? (int64_t)(acc << sh) >> sh : (int64_t)((acc << sh) >> sh);
  }
  if (L.out_type == LT_T_F64) return (double)r;
  if (L.out_type == LT_T_F32) return (double)(float)r;
  int64_t lo, hi;
  lin_out_range(L.out_type, lo, hi);
  return (double)(r < lo ? lo : r > hi ? hi : r);
}
template <class B>
__host__ __device__ inline uint64_t lin_term(int64_t coef, B b) {
  return (uint64_t)coef * (uint64_t)(int64_t)b;
}
__host__ __device__ inline double lin_value(const lt_tile_in& in, int64_t o, int64_t p) {
  const lt_index_lin& L = in.lin;
  uint64_t acc = (uint64_t)L.c0;
  for (int s = 0; s < L.n_bands && s < LT_LIN_MAX_BANDS; s++) {
    const int64_t i = o * in.band_obs_stride + s * in.band_stride + p * in.band_pix_stride;
    switch (L.band_type) {
      case LT_T_I16: acc += lin_term(L.coef[s], ((const int16_t*)in.obs_bands)[i]); break;
      case LT_T_U16: acc += lin_term(L.coef[s], ((const uint16_t*)in.obs_bands)[i]); break;
      case LT_T_U8: acc += lin_term(L.coef[s], ((const uint8_t*)in.obs_bands)[i]); break;
      default: acc += lin_term(L.coef[s], ((const int32_t*)in.obs_bands)[i]); break;
    }
  }
  return lin_store(L, acc);
}

// Whether observation o is valid (not cloud-masked, utils.py:353) at pixel p: the byte mask, the
// mask bit planes, or no mask.
__host__ __device__ inline bool obs_is_valid(const lt_tile_in& in, int64_t o, int64_t p) {
  if (in.obs_valid_bits) return (in.obs_valid_bits[(o >> 5) * in.stride + p] >> (o & 31)) & 1u;
  return in.obs_valid == nullptr || in.obs_valid[o * in.stride + p] != 0;
}

// Value of observation o at pixel p of a tile: the f64 values, the index raster in its stored
// type (float(val), utils.py:357), or the fused load stage's value from the band planes.
// index_type is uniform over a launch: a scalar branch on the GPU.
__host__ __device__ inline double obs_value(const lt_tile_in& in, int64_t o, int64_t p) {
  if (in.obs_bands) return lin_value(in, o, p);
  const int64_t i = o * in.stride + p;
  if (in.obs_index == nullptr) return in.obs_val[i];
  switch (in.index_type) {
    case LT_T_I16: return (double)((const int16_t*)in.obs_index)[i];
    case LT_T_U16: return (double)((const uint16_t*)in.obs_index)[i];
    case LT_T_I32: return (double)((const int32_t*)in.obs_index)[i];
    case LT_T_F32: return (double)((const float*)in.obs_index)[i];
    case LT_T_U8: return (double)((const uint8_t*)in.obs_index)[i];
    case LT_T_U32: return (double)((const uint32_t*)in.obs_index)[i];
    case LT_T_I8: return (double)((const int8_t*)in.obs_index)[i];
    case LT_T_I64: return (double)((const int64_t*)in.obs_index)[i];
    default: return ((const double*)in.obs_index)[i];
  }
}

// Early exit over the starts of a DP column (the reference prices every start, utils.py:618-631;
// starts are visited in decreasing order). For a start i' < i of column j, in exact arithmetic,
//   e(i',j) >= e(i',i-1) + e(i,j)      (least squares on the union of two point sets)
//   OPT[i]  <= OPT[i'] + e(i',i-1) + c (start i' is a candidate of OPT[i])
// so v(i') = e(i',j) + c + OPT[i'] >= e(i,j) + OPT[i]; with c >= 0 (OPT >= 0) also >= e(i,j) + c.
// The bound below holds for the reference's rounded values: eopt >= |opta - OPT_ref[i]|, each of
// the three residuals involved is within kScreen * its sum(y^2) <= SyyAll of the exact one, and
// the factors cover the roundings. Once it exceeds an upper bound on the column minimum, no start
// below i can be (or tie) the minimum.
__host__ __device__ inline double dp_start_bound_slack(double e, double opta, double eopt,
                                                       double c, double slack) {
  const double o = opta - eopt > c ? opta - eopt : c;
  return (e + o) * (1.0 - 0x1p-49) - slack;
}
__host__ __device__ inline double dp_start_bound(double e, double opta, double eopt, double c,
                                                 double SyyAll) {
  return dp_start_bound_slack(e, opta, eopt, c, 4.0 * kScreen * SyyAll * (1.0 + 0x1p-49));
}

// Zero-residual starts. The reference prices start i of column j as fl(fl(e + c) + OPT[i])
// (utils.py:627) with e = 0.0 exactly for 1-2 points (no residuals, utils.py:592-597) and e >= 0
// the emulated dgelsd residual otherwise. When the segment's exact SSE is 0 (collinear points)
// and kZero * Syy < 2^-54 c, e lies below half an ulp of c, so fl(e + c) = c: the start is worth
// fl(c + OPT[i]) like a 1-2 point start, and is exact whenever OPT[i] is.
// kZero bounds the emulated residual of exactly collinear segments: tests/test_screening.py
// measures at most 2^-93 Syy (m <= 64, int16 values, gapped x sets). The a-priori bound (DESIGN.md
// § Screening bounds, tests/test_screening_bounds.py) is eta^2 Syy with eta growing with the
// segment's largest year offset X: at most 2^-84 for X <= 63, but up to 2^-80.2 for X <= 255
// (year spans up to 255 are accepted, lt_abi.hip), so segments reaching past offset 63 use
// kZeroWide instead (zero_bound).
constexpr double kZero = 0x1p-80;
constexpr double kZeroWide = 0x1p-74;
__host__ __device__ inline double zero_bound(int x_max) { return x_max <= 63 ? kZero : kZeroWide; }

// t1 * D == N1^2 exactly (the closed form's numerator m*D*SSE is 0): t1, D and N1 are exact
// integers in binary64 when the values are integers of int16 range (|Sy| < 2^21, Syy < 2^36),
// and each product is split exactly into a double pair.
__host__ __device__ inline bool sse_exact_zero(double t1, double D, double N1) {
  const double p = t1 * D, q = N1 * N1;
  return p == q && __builtin_fma(t1, D, -p) == __builtin_fma(N1, N1, -q);
}

// Tags of inexact OPT values. tag = (b << 8) | t says OPT[k] = g^t(OPT[b]) with g(x) = fl(c + x)
// and b >= 1 (tag < 256: OPT[k] is exact). Two zero-residual starts whose OPT values share a
// base are ordered without knowing OPT[b]: g is non-decreasing for c >= 0, so t <= t' gives
// fl(c + OPT) <= fl(c + OPT'), and strictly increasing while c exceeds the rounding of x + c.
// Returns whether a start of tag `tn` (a smaller start than the one of tag `tg`) is provably
// <= (1), provably > (-1), or neither (0) in value.
__host__ __device__ inline int tag_order(int tn, int tg, double v, double c) {
  if ((tn >> 8) != (tg >> 8)) return 0;
  if ((tn & 255) <= (tg & 255)) return 1;
  return c > 0x1p-50 * __builtin_fabs(v) ? -1 : 0;
}

// segmented_least_squares' DP (utils.py:618-631) with candidate screening.
// For column j every start i is first priced with the closed-form SSE of its segment (exact
// integer sums for integer data); only the starts whose price lies within the error window of
// the column minimum are re-priced with the emulated LAPACK residual, and the first exact
// minimum among them wins — the same argmin and the same OPT bits as pricing every start
// exactly, because a start outside the window is strictly worse than the approximate argmin.
template <int MAXY>
__host__ __device__ inline void dp_screened(int n, const uint8_t* xs, const double* ys, double c,
                                   double* OPT, uint8_t* arg, int& status) {
  double va[MAXY];
  double SyyAll = 0.0;  // sum of y^2 over the points 0..j
  for (int j = 0; j < n; j++) {
    // pass 1: approximate price of every start, i from j down to 0 (incremental sums)
    double Sy = 0.0, Sxy = 0.0, Syy = 0.0;
    int Sx = 0, Sxx = 0;
    double vmin = __builtin_inf(), wmax = 0.0, Hc = __builtin_inf();
    SyyAll += ys[j] * ys[j];
    for (int i = 0; i <= j; i++) va[i] = __builtin_inf();
    for (int i = j; i >= 0; i--) {
      const int xi = xs[i];
      const double yi = ys[i];
      Sx += xi;
      Sxx += xi * xi;
      Sy += yi;
      Sxy += (double)xi * yi;
      Syy += yi * yi;
      const int m = j - i + 1;
      double e = 0.0, w = 0.0;
      if (m >= 3) {
        const double md = (double)m;
        const double D = (double)(m * Sxx - Sx * Sx);
        const double t1 = md * Syy - Sy * Sy;
        const double N1 = md * Sxy - (double)Sx * Sy;
        e = (t1 - N1 * N1 / D) / md;
        if (e < 0.0) e = 0.0;
        w = kScreen * Syy;
      }
      const double v = (e + c) + OPT[i];
      w += 0x1p-50 * __builtin_fabs(v);
      va[i] = v;
      vmin = v < vmin ? v : vmin;
      wmax = w > wmax ? w : wmax;
      Hc = v + w < Hc ? v + w : Hc;
      if (m >= 3 && c >= 0.0 && dp_start_bound(e, OPT[i], 0.0, c, SyyAll) > Hc) break;
    }
    // pass 2: exact price for the starts inside the window, first exact minimum wins
    const double lim = vmin + 2.0 * wmax;
    double best = 0.0;
    int bi = -1;
    for (int i = 0; i <= j; i++) {
      if (!(va[i] <= lim)) continue;
      const int m = j - i + 1;
      double e = 0.0;
      if (m >= 3) {
        double sm, sb, ssr;
        int rc = lstsq_xint(
            m, [&](int k) { return (int)xs[i + k]; }, [&](int k) { return ys[i + k]; }, false,
            true, sm, sb, ssr);
        if (rc < 0) status |= LT_ST_NUMERIC;
        e = ssr;
      }
      const double v = (e + c) + OPT[i];
      if (bi < 0 || v < best) {
        best = v;
        bi = i;
      }
    }
    OPT[j + 1] = best;
    arg[j] = (uint8_t)bi;
  }
}

// The same DP with every OPT value kept only approximately, together with a rigorous bound
// E[j] >= |OPTa[j] - OPT[j]|. Column j is decided without any LAPACK emulation when one start's
// upper bound lies strictly below every other start's lower bound (then it is the unique exact
// minimum). Otherwise the column is marked ambiguous, carries the approximate minimum and the
// width of the uncertainty forward, and the DP goes on. Only the backtracked path matters for
// the result: if it crosses no ambiguous column, every vertex is exact; otherwise the function
// returns false and the pixel is re-run with dp_screened (exact OPT) by the resolve kernel.
template <int MAXY>
__host__ __device__ inline bool dp_lazy(int n, const uint8_t* xs, const double* ys, double c,
                                        uint8_t* arg, uint64_t* amb_out = nullptr) {
  double OPTa[MAXY + 1], E[MAXY + 1];
  int TG[MAXY + 1];  // tags (tag_order) of the OPT values
  uint64_t amb = 0;
  OPTa[0] = 0.0;
  E[0] = 0.0;
  TG[0] = 0;
  // integer values of int16 range: the closed form's sums are exact (sse_exact_zero)
  bool intdata = true;
  for (int k = 0; k < n; k++)
    intdata = intdata && ys[k] == (double)(int)ys[k] && ys[k] >= -32768.0 && ys[k] <= 32767.0;
  const bool zero_ok = c > 0.0;
  double SyyAll = 0.0;  // sum of y^2 over the points 0..j (early exit, as in dp_screened)
  for (int j = 0; j < n; j++) {
    SyyAll += ys[j] * ys[j];
    double Sy = 0.0, Sxy = 0.0, Syy = 0.0;
    int Sx = 0, Sxx = 0;
    // Exact candidates (zero-residual start on an exact OPT) are computed with the reference's
    // own operations, so their value IS the reference's; the others carry an interval
    // [v - w, v + w] around the reference value. Zero-residual starts on inexact OPT values of
    // one base form a group whose best member is known exactly (tag_order); only that member
    // enters the interval trackers, at the end of the column.
    const double inf = __builtin_inf();
    double Ve = inf;                   // min exact value; ie = first start attaining it
    double Hi = inf, Li1 = inf, Li2 = inf, vHi = 0.0, wHi = 0.0, vbest = inf;
    int ie = -1, iHi = -1, ibest = -1, iL1 = -2, tHi = -1;
    double gv = 0.0, gw = 0.0;
    int gi = -1, gtag = 0;
    auto track = [&](int i, double v, double w, int ntag) {
      const double lo = v - w, hi = v + w;
      if (hi <= Hi) {
        Hi = hi;
        iHi = i;
        vHi = v;
        wHi = w;
        tHi = ntag;
      }
      if (lo <= Li1) {  // the two smallest lower ends (equal ones count twice)
        Li2 = Li1;
        Li1 = lo;
        iL1 = i;
      } else if (lo < Li2) {
        Li2 = lo;
      }
    };
    for (int i = j; i >= 0; i--) {
      const int xi = xs[i];
      const double yi = ys[i];
      Sx += xi;
      Sxx += xi * xi;
      Sy += yi;
      Sxy += (double)xi * yi;
      Syy += yi * yi;
      const int m = j - i + 1;
      double e = 0.0, ws = 0.0;
      bool zr = m <= 2;
      if (m >= 3) {
        const double md = (double)m;
        const double D = (double)(m * Sxx - Sx * Sx);
        const double t1 = md * Syy - Sy * Sy;
        const double N1 = md * Sxy - (double)Sx * Sy;
        e = (t1 - N1 * N1 / D) / md;
        if (e < 0.0) e = 0.0;
        ws = kScreen * Syy;
        if (zero_ok && intdata && e <= ws && zero_bound(xs[j]) * Syy < 0x1p-54 * c &&
            sse_exact_zero(t1, D, N1)) {
          zr = true;
          e = 0.0;
          ws = 0.0;
        }
      }
      const double v = (e + c) + OPTa[i];
      bool tracked = true;
      if (zr && E[i] == 0.0) {
        if (v <= Ve) {
          Ve = v;
          ie = i;
        }
      } else if (zr && zero_ok) {
        const double w = E[i] + 0x1p-50 * __builtin_fabs(v);
        const int ord = gi < 0 ? 1 : tag_order(TG[i], gtag, v, c);
        if (ord > 0) {  // the group's new best (i descends: the smaller start, value <=)
          gi = i;
          gtag = TG[i];
          gv = v;
          gw = w;
        } else if (ord < 0) {
          tracked = false;  // strictly above the group's best: never the first minimum
        } else {
          track(i, v, w, TG[i] + 1);
        }
      } else {
        track(i, v, E[i] + ws + 0x1p-50 * __builtin_fabs(v), -1);
      }
      if (tracked && v <= vbest) {  // i descends: "<=" keeps the smaller start on equal values
        vbest = v;
        ibest = i;
      }
      double Hc = Hi < Ve ? Hi : Ve;
      if (gi >= 0 && gv + gw < Hc) Hc = gv + gw;
      if (m >= 3 && c >= 0.0 && dp_start_bound(e, OPTa[i], E[i], c, SyyAll) > Hc) break;
    }
    if (gi >= 0) track(gi, gv, gw, gtag + 1);
    const double H = Hi < Ve ? Hi : Ve;  // the exact minimum lies in [min lower bound, H]
    if (Li1 > H) {  // no interval reaches H: the exact candidates decide, bit-exactly
      arg[j] = (uint8_t)ie;
      OPTa[j + 1] = Ve;
      E[j + 1] = 0.0;
      TG[j + 1] = 0;
    } else if (iL1 == iHi && Li2 > H && Ve > H) {  // one start lies below all others
      arg[j] = (uint8_t)iHi;
      OPTa[j + 1] = vHi;
      E[j + 1] = wHi;
      // a zero-residual start adds c to its OPT value's tag; any other starts a new base
      TG[j + 1] = tHi >= 0 ? tHi : (j + 1) << 8;
    } else {
      TG[j + 1] = (j + 1) << 8;
      amb |= 1ull << j;
      arg[j] = (uint8_t)ibest;
      OPTa[j + 1] = vbest;
      const double L = Li1 < Ve ? Li1 : Ve;
      E[j + 1] = (H - L) * (1.0 + 0x1p-40) + 0x1p-50 * __builtin_fabs(vbest);
    }
  }
  if (amb_out) *amb_out = amb;
  for (int j = n - 1; j >= 0; j = arg[j] - 1)
    if ((amb >> j) & 1) return false;
  return true;
}

// Returns false (and writes nothing final) when LAZY and the pixel needs the exact-OPT DP.
template <int MAXY, bool LAZY>
__host__ __device__ bool analyze_pixel(const DevScene& S, const lt_params& P, const lt_tile_in& in,
                                       const lt_tile_out& out, int64_t p) {
  const int Y = S.n_years;
  const int64_t is = in.stride, os = out.stride;
  int status = LT_ST_OK;

  // ---- pick_winners: per year slot, first valid obs (input order) at minimal |days| ----
  double val[MAXY];
  uint8_t slot[MAXY];
  int T = 0;
  for (int y = 0; y < Y; y++) {
    int best = -1, bd = 0x7fffffff;
    const int k1 = S.slot_begin[y + 1];
    for (int k = S.slot_begin[y]; k < k1; k++) {
      const int o = S.order[k];
      const bool ok = obs_is_valid(in, o, p);
      if (ok && S.dist[k] < bd) {
        bd = S.dist[k];
        best = o;
      }
    }
    if (out.winner) out.winner[(int64_t)y * os + p] = (int16_t)best;
    if (best >= 0) {
      if ((S.feb29_mask >> y) & 1) status |= LT_ST_FEB29;
      val[T] = obs_value(in, (int64_t)best, p);
      slot[T] = (uint8_t)y;
      T++;
    }
  }
  if (out.n_years) out.n_years[p] = T;
  const int y0 = T > 0 ? S.year[slot[0]] : 0;

  uint64_t spike_m = 0;  // bits over the T-point series
  const bool ok = T >= 2;
  if (T == 0) status |= LT_ST_EMPTY;
  if (T == 1) status |= LT_ST_SINGLE_YEAR;
  const double nan = __builtin_nan("");

  // per-year outputs of absent years (and of every year when the reference raises)
  {
    int t = 0;
    for (int y = 0; y < Y; y++) {
      const bool present = t < T && slot[t] == y;
      const int64_t q = (int64_t)y * os + p;
      if (!present || !ok) {
        if (out.val_raw) out.val_raw[q] = present ? val[t] : nan;
        if (out.val_fit) out.val_fit[q] = nan;
        if (out.fit_m) out.fit_m[q] = nan;
        if (out.fit_b) out.fit_b[q] = nan;
        if (out.right_m) out.right_m[q] = nan;
        if (out.right_b) out.right_b[q] = nan;
        if (out.spike) out.spike[q] = 0;
        if (out.vertex) out.vertex[q] = 0;
      }
      if (present) t++;
    }
  }

  RuleState rs;
  rs.reset(P.n_rules);

  if (ok) {
    // ---- despike (utils.py:556-582) ----
    const double avg = np_sum(T, [&](int i) { return val[i]; }) / (double)T;
    const double sd = __builtin_sqrt(np_sum(T, [&](int i) {
                                       double d = avg - val[i];
                                       return d * d;
                                     }) /
                                     (double)T);
    double last_good = val[0];
    for (int i = 1; i < T - 1; i++) {
      const double xv = val[i - 1], yv = val[i], zv = val[i + 1];
      const bool mono = (xv <= yv && yv <= zv) || (xv >= yv && yv >= zv);
      if (!mono && (__builtin_fabs(yv - xv) > sd && __builtin_fabs(yv - zv) > sd) &&
          yv != last_good) {
        spike_m |= 1ull << i;
      } else {
        last_good = yv;
      }
    }
    // ---- dropna: the non-spike series (x = year offset) ----
    double ys[MAXY];
    uint8_t xs[MAXY];
    int n = 0;
    for (int i = 0; i < T; i++) {
      if ((spike_m >> i) & 1) continue;
      xs[n] = (uint8_t)(S.year[slot[i]] - y0);
      ys[n] = val[i];
      n++;
    }
    // ---- segmented least squares DP (utils.py:618-631) ----
#ifdef LT_HOST_DIAG
    lt_host_diag_series(p, n, xs, ys);  // host diagnostics (tests/native): the DP's input series
#endif
    uint8_t arg[MAXY];
    if constexpr (LAZY) {
      if (!dp_lazy<MAXY>(n, xs, ys, P.line_cost, arg)) return false;
    } else {
      double OPT[MAXY + 1];
      OPT[0] = 0.0;
      dp_screened<MAXY>(n, xs, ys, P.line_cost, OPT, arg, status);
    }
    // ---- find_segments: starts of the optimal segments + the last point ----
    uint64_t vnon = 1ull << (n - 1);  // over non-spike indices
    for (int j = n - 1; j >= 0; j = arg[j] - 1) vnon |= 1ull << arg[j];

    // ---- vertices2eqns + eqns2fitted_points + labels, walking the full series ----
    double cm = 0.0, cb = 0.0;  // eqn of the current (most recent) vertex
    int k = 0;                  // non-spike index
    double left_fit = 0.0;
    int32_t left_year = y0;
    for (int i = 0; i < T; i++) {
      const bool sp = (spike_m >> i) & 1;
      bool is_v = false;
      const double pm = cm, pb = cb;  // left eqn = previous point's right eqn
      if (!sp) {
        if ((vnon >> k) & 1) {
          is_v = true;
          const uint64_t later = vnon & ~((2ull << k) - 1);
          if (later) {  // not the last vertex: LS over [k, next vertex] (label-inclusive)
            const int k2 = __builtin_ctzll(later);
            double sm, sb, ssr;
            int rc = lstsq_xint(
                k2 - k + 1, [&](int q) { return (int)xs[k + q]; },
                [&](int q) { return ys[k + q]; }, true, false, sm, sb, ssr);
            if (rc < 0) status |= LT_ST_NUMERIC;
            cm = sm;
            cb = sb;
          }  // last vertex reuses the previous vertex's eqn (utils.py:662)
        }
        k++;
      }
      const int32_t yr = S.year[slot[i]];
      const double x = (double)(yr - y0);
      double fv, fmv, fbv;
      if (i == 0 || (pm == cm && pb == cb)) {
        fv = (cm * x) + cb;
        fmv = cm;
        fbv = cb;
      } else {
        const double fl = (pm * x) + pb;
        const double fr = (cm * x) + cb;
        const double raw = sp ? nan : val[i];
        if (__builtin_fabs(fl - raw) <= __builtin_fabs(fr - raw)) {
          fv = fl; fmv = pm; fbv = pb;
        } else {
          fv = fr; fmv = cm; fbv = cb;
        }
      }
      const int64_t q = (int64_t)slot[i] * os + p;
      if (out.val_raw) out.val_raw[q] = val[i];
      if (out.val_fit) out.val_fit[q] = fv;
      if (out.fit_m) out.fit_m[q] = fmv;
      if (out.fit_b) out.fit_b[q] = fbv;
      if (out.right_m) out.right_m[q] = cm;
      if (out.right_b) out.right_b[q] = cb;
      if (out.spike) out.spike[q] = sp ? 1 : 0;
      if (out.vertex) out.vertex[q] = is_v ? 1 : 0;

      // parse_disturbances (classes.py:156-176): the first point is the first left vertex
      if (i == 0) {
        left_fit = fv;
        left_year = yr;
      } else if (is_v) {
        const int32_t on = left_year;
        const int32_t du = yr - left_year;
        const double init = left_fit;
        const double mag = left_fit - fv;
        left_fit = fv;
        left_year = yr;
        rs.offer(P, on, du, init, mag, status);
      }
    }
  }

  rs.write(P, out, p);
  if (out.status) out.status[p] = status;
  return true;
}

// Label stage alone (change_labeling on an existing trendline): per slot y, val_fit / vertex /
// present planes; the first present point is the first left vertex (classes.py:163-164).
__host__ __device__ inline void label_pixel(const int32_t* year, int Y, const lt_params& P,
                                   const lt_label_in& in, const lt_tile_out& out, int64_t p) {
  const int64_t is = in.stride;
  int status = LT_ST_OK;
  RuleState rs;
  rs.reset(P.n_rules);
  bool first = true;
  double left_fit = 0.0;
  int32_t left_year = 0;
  for (int y = 0; y < Y; y++) {
    const int64_t q = (int64_t)y * is + p;
    if (in.present && !in.present[q]) continue;
    const double fv = in.val_fit[q];
    if (first) {
      first = false;
      left_fit = fv;
      left_year = year[y];
      continue;
    }
    if (!in.vertex[q]) continue;
    rs.offer(P, left_year, year[y] - left_year, left_fit, left_fit - fv, status);
    left_fit = fv;
    left_year = year[y];
  }
  rs.write(P, out, p);
  if (out.status) out.status[p] = status;
}

}  // namespace lt
