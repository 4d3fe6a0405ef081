// Host-side harness for the device code (land_trendr_amd/csrc/lt_lapack.h, lt_pixel.h).
// TEST INFRASTRUCTURE: compiles the exact __host__ __device__ code the kernels run, for the CPU,
// so tests/test_lapack_emulation.py and tests/test_kernel_host.py can compare it with the oracle
// and the reference goldens without a GPU. Built by __graft_entry__.build() into
// tests/native/build/liblt_hostcheck.so. Not part of the product (which has no CPU path).
#include <string.h>

// diagnostics hook of lt_pixel.h analyze_pixel: the compacted (non-spike) series the DP takes
#define LT_HOST_DIAG 1
static int g_diag_n = -1;
static uint8_t g_diag_xs[64];
static double g_diag_ys[64];
static void lt_host_diag_series(long long, int n, const uint8_t* xs, const double* ys) {
  g_diag_n = n;
  for (int k = 0; k < n && k < 64; k++) {
    g_diag_xs[k] = xs[k];
    g_diag_ys[k] = ys[k];
  }
}
#include "../../land_trendr_amd/csrc/lt_pixel.h"

extern "C" int ltx_lstsq(int m, const double* x, const double* y, int want_solution,
                         double* out3) {
  double s, c, r;
  int rc = lt::lstsq_segment(m, [&](int k) { return x[k]; }, [&](int k) { return y[k]; },
                             want_solution != 0, s, c, r);
  out3[0] = s;
  out3[1] = c;
  out3[2] = r;
  return rc;
}

extern "C" double ltx_nrm2(int n, const double* x) {
  return lt::nrm2(n, [&](int k) { return x[k]; });
}

// The kernel's per-pixel pipeline run over a host tile (same structs as lt_analyze_tile).
extern "C" int ltx_analyze_tile(const lt_scene* sc, const lt_params* prm, const lt_tile_in* in,
                                const lt_tile_out* out) {
  static lt::DevScene S;
  memset(&S, 0, sizeof S);
  S.n_obs = sc->n_obs;
  S.n_years = sc->n_years;
  for (int y = 0; y < sc->n_years; y++) {
    S.year[y] = sc->year[y];
    if (sc->feb29_bad && sc->feb29_bad[y]) S.feb29_mask |= 1ull << y;
  }
  for (int y = 0; y <= sc->n_years; y++) S.slot_begin[y] = sc->n_years ? sc->slot_begin[y] : 0;
  for (int k = 0; k < sc->n_obs; k++) {
    S.order[k] = sc->order[k];
    S.dist[k] = sc->dist[k];
  }
  int deferred = 0;  // same two stages as the GPU: lazy DP, exact-OPT DP for deferred pixels
  for (int64_t p = 0; p < in->n_pix; p++) {
    bool done = S.n_years <= 32 ? lt::analyze_pixel<32, true>(S, *prm, *in, *out, p)
                                : lt::analyze_pixel<64, true>(S, *prm, *in, *out, p);
    if (done) continue;
    deferred++;
    if (S.n_years <= 32) lt::analyze_pixel<32, false>(S, *prm, *in, *out, p);
    else lt::analyze_pixel<64, false>(S, *prm, *in, *out, p);
  }
  return deferred;
}

// Diagnostics: the lazy DP on one compacted series; returns the ambiguous-column mask.
extern "C" uint64_t ltx_dp_lazy(int n, const uint8_t* xs, const double* ys, double c,
                                uint8_t* arg, int* deferred) {
  uint64_t amb = 0;
  *deferred = !lt::dp_lazy<64>(n, xs, ys, c, arg, &amb);
  return amb;
}

// The exact-OPT DP (dp_screened: LAPACK-emulated residual for every start in the window) on one
// compacted series: the argmin of every column.
extern "C" int ltx_dp_exact(int n, const uint8_t* xs, const double* ys, double c, uint8_t* arg) {
  double OPT[65];
  OPT[0] = 0.0;
  int status = 0;
  lt::dp_screened<64>(n, xs, ys, c, OPT, arg, status);
  return status;
}

// The integer-x fused variant (lstsq_xint) on integer x given as doubles.
extern "C" int ltx_lstsq_xint(int m, const double* x, const double* y, int need_solution,
                              int need_ssr, double* out3) {
  double s, c, r;
  int rc = lt::lstsq_xint(m, [&](int k) { return (int)x[k]; }, [&](int k) { return y[k]; },
                          need_solution != 0, need_ssr != 0, s, c, r);
  out3[0] = s;
  out3[1] = c;
  out3[2] = r;
  return rc;
}

// dnrm2 on binary64 pairs; *slow = 1 when the caller would fall back to nrm2()
extern "C" double ltx_nrm2_dd(int n, const double* x, int* slow) {
  bool s = false;
  const double r = lt::nrm2_dd(n, [&](int k) { return x[k]; }, s);
  *slow = s;
  return r;
}

// x87 sqrt-then-store of hi + lo: out2 = {binary64 path, integer soft-float80 path}; returns slow
extern "C" int ltx_sqrt_pair(double hi, double lo, double* out2) {
  bool s = false;
  out2[0] = lt::xdd_sqrt_to_double(hi, lo, s);
  out2[1] = lt::f80_sqrt_to_double(lt::xdd_to_f80(lt::xdd{hi, lo}));
  return s;
}

// x-set table keys: round trip of every slot; returns the number of mismatches
extern "C" int ltx_xset_roundtrip(int* n_valid) {
  int bad = 0, nv = 0;
  for (int idx = 0; idx < lt::kXtSize; idx++) {
    int m = 0, xs[64];
    if (!lt::xset_of_key(idx, m, xs)) continue;
    nv++;
    bad += lt::xset_key(m, [&](int k) { return xs[k]; }) != idx;
  }
  *n_valid = nv;
  return bad;
}

// lsq_apply_small (the vertex fits' straight-line path, m <= 4) against lsq_apply on the same
// factorisation: out4 = {small slope, small intercept, general slope, general intercept};
// returns the two return codes packed as small * 16 + general (each offset by 8)
extern "C" int ltx_lsq_small_vs_general(int m, const double* x, const double* y, double* out4) {
  lt::lsq_xf f;
  auto X = [&](int k) { return (int)x[k]; };
  auto Y = [&](int k) { return y[k]; };
  lt::lsq_factor(m, X, f);
  double s0, c0, s1, c1, r1;
  const int a = lt::lsq_apply_small(f, X, Y, s0, c0);
  const int b = lt::lsq_apply(f, X, Y, true, false, s1, c1, r1);
  out4[0] = s0;
  out4[1] = c0;
  out4[2] = s1;
  out4[3] = c1;
  return (a + 8) * 16 + (b + 8);
}

// lt_pixel.h RuleCands against the full replay: n disturbances (onset, duration, exact init and
// magnitude, half-widths of the intervals the candidate pass sees) offered to rule R. Returns 1
// when replaying RuleState1 over the candidate set alone gives the full replay's winner (every
// field bit-equal and the same status), 0 otherwise; *n_cand = size of the candidate set.
extern "C" int ltx_rule_cands(int n, const int32_t* on, const int32_t* du, const double* init,
                              const double* mag, const double* w_init, const double* w_mag,
                              const lt_rule* R, int pre_mode, int* n_cand) {
  lt::RuleState1 full, part;
  lt::RuleCands cand;
  int st_full = 0, st_cand = 0, st_part = 0;
  for (int i = 0; i < n; i++) {
    full.offer(*R, pre_mode, on[i], du[i], init[i], mag[i], st_full);
    cand.offer(*R, pre_mode, on[i], du[i], init[i] - w_init[i], init[i] + w_init[i],
               mag[i] - w_mag[i], mag[i] + w_mag[i], 1ull << i, st_cand);
  }
  for (int i = 0; i < n; i++)
    if ((cand.G >> i) & 1) part.offer(*R, pre_mode, on[i], du[i], init[i], mag[i], st_part);
  *n_cand = __builtin_popcountll(cand.G);
  auto same = [](double a, double b) { return __builtin_memcmp(&a, &b, sizeof a) == 0; };
  return full.have == part.have && full.on == part.on && full.du == part.du &&
         same(full.mag, part.mag) && same(full.init, part.init) &&
         (n == 0 || st_cand == st_full);
}

// The DP's input series (after pick_winners, despike and dropna) of the last pixel
// ltx_analyze_tile processed: returns n (-1: none reached the DP), fills xs / ys.
extern "C" int ltx_last_series(uint8_t* xs, double* ys) {
  for (int k = 0; k < g_diag_n; k++) {
    xs[k] = g_diag_xs[k];
    ys[k] = g_diag_ys[k];
  }
  const int n = g_diag_n;
  g_diag_n = -1;
  return n;
}
