/*
 * lt_oracle.c — CPU restatement of the reference per-pixel path. TEST INFRASTRUCTURE (see header).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; every fused multiply-add below is an explicit
 * fma() because the reference's OpenBLAS SkylakeX kernels fuse exactly there).
 * The x87 part of OpenBLAS dnrm2 is restated with the host's own 80-bit long double
 * (x86-64 gcc: long double = x87 extended, 64-bit significand), independently of the device's
 * soft-float80 in land_trendr_amd/csrc/lt_lapack.h — the two cross-check each other.
 */
#include "lt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#if !defined(__x86_64__) && !defined(__i386__)
#error "the oracle restates x87 dnrm2 with long double; build it on x86"
#endif

/* ------------------------------------------------------------------------------------------ */
/* numpy pairwise sum: np.sum over a contiguous float64 array, n <= 128.          */
/* ------------------------------------------------------------------------------------------ */
static double np_pairwise_sum(int n, const double* a) {
  if (n < 8) {
    double r = 0.0;  /* numpy starts from -0.0 for n<8? it starts res = 0. then adds */
    for (int i = 0; i < n; i++) r += a[i];
    return r;
  }
  double r[8];
  for (int k = 0; k < 8; k++) r[k] = a[k];
  int i;
  for (i = 8; i < n - (n % 8); i += 8)
    for (int k = 0; k < 8; k++) r[k] += a[i + k];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += a[i];
  return res;
}

/* np.std(time_series) at utils.py:566 → pandas nanops.nanstd(ddof=0): sqrt(nanvar). */
double lto_std(int n, const double* v) {
  double sq[LT_MAX_YEARS];
  double avg = np_pairwise_sum(n, v) / (double)n;
  for (int i = 0; i < n; i++) {
    double d = avg - v[i];
    sq[i] = d * d;
  }
  return sqrt(np_pairwise_sum(n, sq) / (double)n);
}

/* ------------------------------------------------------------------------------------------ */
/* BLAS/LAPACK pieces reached by dgelsd for an m x 2 problem.                 */
/* ------------------------------------------------------------------------------------------ */

/* OpenBLAS dnrm2_k SkylakeX (x87): four 80-bit accumulators, 8-element blocks (A.3). */
static double blas_dnrm2(int n, const double* x) {
  if (n <= 0) return 0.0;
  if (n == 1) return fabs(x[0]);
  long double a[4] = {0.0L, 0.0L, 0.0L, 0.0L};
  int n8 = n & ~7, j;
  for (j = 0; j < n8; j++) {
    long double xv = (long double)x[j];
    a[j & 3] += xv * xv;
  }
  for (; j < n; j++) {
    long double xv = (long double)x[j];
    a[0] += xv * xv;
  }
  long double t = ((a[0] + a[2]) + a[1]) + a[3];
  return (double)sqrtl(t);
}

/* OpenBLAS dgemv_t SkylakeX, one column, alpha 1, beta 0: y = a . v (A.4). */
static double blas_dgemv_t1(int m, const double* a, const double* v) {
  int m3 = m & 3, m1 = m - m3;
  double y = 0.0;
  if (m1 > 0) {
    double L[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = 0; i < m1; i++) {
      double p = a[i] * v[i];
      L[i & 3] = L[i & 3] + p;
    }
    double r = (L[0] + L[2]) + (L[1] + L[3]);
    y = fma(r, 1.0, y);
  }
  if (m3 == 1) {
    y = fma(a[m1], v[m1], y);
  } else if (m3 == 2) {
    y = y + fma(a[m1], v[m1], a[m1 + 1] * v[m1 + 1]);
  } else if (m3 == 3) {
    y = y + fma(a[m1 + 2], v[m1 + 2], fma(a[m1], v[m1], a[m1 + 1] * v[m1 + 1]));
  }
  return y;
}

/* DLARF side L on one column c[0..m-1] with v (v[0] = 1): c -= tau * v * (v' c) (A.2). */
static void lapack_dlarf1(int m, const double* v, double tau, double* c) {
  if (tau == 0.0) return;
  int lastv = m;
  while (lastv > 0 && v[lastv - 1] == 0.0) lastv--;
  int any = 0;
  for (int i = 0; i < lastv; i++)
    if (c[i] != 0.0) { any = 1; break; }
  if (!any) return;
  double w = blas_dgemv_t1(lastv, c, v);
  double s = (-tau) * w;
  for (int i = 0; i < lastv; i++) c[i] = fma(s, v[i], c[i]);
}

/* DLAPY2. */
static double lapack_dlapy2(double x, double y) {
  double xa = fabs(x), ya = fabs(y);
  double w = xa > ya ? xa : ya;
  double z = xa < ya ? xa : ya;
  if (z == 0.0) return w;
  double t = z / w;
  return w * sqrt(1.0 + t * t);
}

/* DLARFG on (alpha, xs[0..n-2]); scales xs in place into v[1..], returns tau, *alpha <- beta. */
static double lapack_dlarfg(int n, double* alpha, double* xs) {
  if (n <= 1) return 0.0;
  double xn = blas_dnrm2(n - 1, xs);
  if (xn == 0.0) return 0.0;
  double beta = -copysign(lapack_dlapy2(*alpha, xn), *alpha);
  double tau = (beta - *alpha) / beta;
  double s = 1.0 / (*alpha - beta);
  for (int i = 0; i < n - 1; i++) xs[i] = xs[i] * s;
  *alpha = beta;
  return tau;
}

static double fsign(double a, double b) { return copysign(fabs(a), b); }

/* DLASV2 (LAPACK 3.x), literal (A.6). */
static void lapack_dlasv2(double f, double g, double h, double* ssmin, double* ssmax,
                          double* snr, double* csr, double* snl, double* csl) {
  const double eps = 0x1p-53;
  double ft = f, fa = fabs(ft), ht = h, ha = fabs(h);
  int pmax = 1;
  int swap = ha > fa;
  if (swap) {
    pmax = 3;
    double tmp = ft; ft = ht; ht = tmp;
    tmp = fa; fa = ha; ha = tmp;
  }
  double gt = g, ga = fabs(gt);
  double clt, crt, slt, srt, smin, smax;
  if (ga == 0.0) {
    smin = ha; smax = fa;
    clt = 1.0; crt = 1.0; slt = 0.0; srt = 0.0;
  } else {
    int gasmal = 1;
    if (ga > fa) {
      pmax = 2;
      if ((fa / ga) < eps) {
        gasmal = 0;
        smax = ga;
        if (ha > 1.0) smin = fa / (ga / ha);
        else smin = (fa / ga) * ha;
        clt = 1.0;
        slt = ht / gt;
        srt = 1.0;
        crt = ft / gt;
      }
    }
    if (gasmal) {
      double d = fa - ha;
      double l = (d == fa) ? 1.0 : d / fa;
      double m = gt / ft;
      double t = 2.0 - l;
      double mm = m * m, tt = t * t;
      double s = sqrt(tt + mm);
      double r = (l == 0.0) ? fabs(m) : sqrt(l * l + mm);
      double a = 0.5 * (s + r);
      smin = ha / a;
      smax = fa * a;
      if (mm == 0.0) {
        if (l == 0.0) t = fsign(2.0, ft) * fsign(1.0, gt);
        else t = gt / fsign(d, ft) + m / t;
      } else {
        t = (m / (s + t) + m / (r + l)) * (1.0 + a);
      }
      l = sqrt(t * t + 4.0);
      crt = 2.0 / l;
      srt = t / l;
      clt = (crt + srt * m) / a;
      slt = ((ht / ft) * srt) / a;
    }
  }
  if (swap) { *csl = srt; *snl = crt; *csr = slt; *snr = clt; }
  else      { *csl = clt; *snl = slt; *csr = crt; *snr = srt; }
  double tsign = 1.0;
  if (pmax == 1) tsign = fsign(1.0, *csr) * fsign(1.0, *csl) * fsign(1.0, f);
  if (pmax == 2) tsign = fsign(1.0, *snr) * fsign(1.0, *csl) * fsign(1.0, g);
  if (pmax == 3) tsign = fsign(1.0, *snr) * fsign(1.0, *snl) * fsign(1.0, h);
  *ssmax = fsign(smax, tsign);
  *ssmin = fsign(smin, tsign * fsign(1.0, f) * fsign(1.0, h));
}

/* DLALSD for N = 2 (DLASDQ → DBDSQR 2x2 → solve → back-transform), A.5.
 * Returns the rank (numpy reports residuals only for rank 2), or -1 on an unemulated path. */
static int lapack_dlalsd2(double d1, double d2, double e, double b1, double b2, double rcond,
                          double* x0, double* x1) {
  const double eps = 0x1p-53, unfl = 0x1p-1022;
  double rcnd = (rcond > 0.0 && rcond < 1.0) ? rcond : eps;
  double org = fabs(d1);
  if (fabs(d2) > org || isnan(d2)) org = fabs(d2);
  if (fabs(e) > org || isnan(e)) org = fabs(e);
  if (org == 0.0) { *x0 = 0.0; *x1 = 0.0; return 0; }
  /* DLASCL multi-step scaling only triggers near under/overflow: not emulated. */
  if (!(org > 0x1p-900 && org < 0x1p900)) return -1;
  double mul = 1.0 / org;
  d1 *= mul; d2 *= mul; e *= mul;
  double vt00 = 1.0, vt01 = 0.0, vt10 = 0.0, vt11 = 1.0;
  /* DBDSQR: tolerance and threshold (relative accuracy branch). */
  const double tolmul = 98.70149282610821; /* max(10, min(100, eps^(-1/8))), see tests */
  double tol = tolmul * eps;
  double sminoa = fabs(d1);
  if (sminoa != 0.0) {
    double mu = fabs(d2) * (sminoa / (sminoa + fabs(e)));
    if (mu < sminoa) sminoa = mu;
  }
  sminoa = sminoa / sqrt(2.0);
  double thresh = tol * sminoa;
  double floor_ = 6.0 * (2.0 * (2.0 * unfl));
  if (floor_ > thresh) thresh = floor_;
  if (fabs(e) > thresh) {
    double ssmin, ssmax, snr, csr, snl, csl;
    lapack_dlasv2(d1, e, d2, &ssmin, &ssmax, &snr, &csr, &snl, &csl);
    d1 = ssmax; d2 = ssmin;
    /* DROT on the VT rows (ncvt = 2) and on the rhs (ncc = 1). */
    double a0 = vt00, b0 = vt10;
    vt00 = fma(csr, a0, snr * b0);
    vt10 = fma(csr, b0, -(snr * a0));
    double a1 = vt01, bb1 = vt11;
    vt01 = fma(csr, a1, snr * bb1);
    vt11 = fma(csr, bb1, -(snr * a1));
    double c0 = b1, c1 = b2;
    b1 = fma(csl, c0, snl * c1);
    b2 = fma(csl, c1, -(snl * c0));
  }
  /* make singular values non-negative */
  if (d1 < 0.0) { d1 = -d1; vt00 = -vt00; vt01 = -vt01; }
  if (d2 < 0.0) { d2 = -d2; vt10 = -vt10; vt11 = -vt11; }
  /* DBDSQR sorts descending ... */
  if (d2 > d1) {
    double t = d1; d1 = d2; d2 = t;
    t = vt00; vt00 = vt10; vt10 = t;
    t = vt01; vt01 = vt11; vt11 = t;
    t = b1; b1 = b2; b2 = t;
  }
  /* ... and DLASDQ re-sorts ascending. */
  if (d2 < d1) {
    double t = d1; d1 = d2; d2 = t;
    t = vt00; vt00 = vt10; vt10 = t;
    t = vt01; vt01 = vt11; vt11 = t;
    t = b1; b1 = b2; b2 = t;
  }
  /* solve: zero the negligible singular values, scale the rest */
  double dmax = fabs(d1);
  if (fabs(d2) > dmax) dmax = fabs(d2);
  double tol2 = rcnd * dmax;
  int rank = 0;
  if (d1 <= tol2) b1 = 0.0;
  else { double q = 1.0 / d1; b1 = b1 * q; rank++; }
  if (d2 <= tol2) b2 = 0.0;
  else { double q = 1.0 / d2; b2 = b2 * q; rank++; }
  double s0 = fma(vt10, b2, vt00 * b1);
  double s1 = fma(vt11, b2, vt01 * b1);
  *x0 = s0 * mul;
  *x1 = s1 * mul;
  return rank;
}

/* np.linalg.lstsq(A=[x|1], y) via dgelsd (utils.py:594-597). */
int lto_lstsq(int m, const double* x, const double* y, double* slope, double* icpt,
              double* ssr) {
  if (m < 2 || m > LT_MAX_OBS) return -2;
  double v1[LT_MAX_OBS], c[LT_MAX_OBS], b[LT_MAX_OBS];
  double rcond = 0x1p-52 * (double)(m > 2 ? m : 2);
  /* DGELSD: B == 0 returns the zero solution with rank 0 (numpy: no residuals → 0.0);
   * B or A outside [SMLNUM, BIGNUM] = [2^-970, 2^970] would be rescaled (not emulated). */
  double bnrm = 0.0, anrm = 1.0;
  for (int i = 0; i < m; i++) {
    if (fabs(y[i]) > bnrm) bnrm = fabs(y[i]);
    if (fabs(x[i]) > anrm) anrm = fabs(x[i]);
  }
  if (bnrm == 0.0) { *slope = 0.0; *icpt = 0.0; *ssr = 0.0; return 0; }
  if (bnrm < 0x1p-970 || bnrm > 0x1p970 || anrm > 0x1p970) return -1;
  /* H1 on column 1 */
  double alpha = x[0];
  for (int i = 1; i < m; i++) v1[i] = x[i];
  v1[0] = 1.0;
  double tau1 = lapack_dlarfg(m, &alpha, v1 + 1);
  double beta1 = alpha;
  for (int i = 0; i < m; i++) { c[i] = 1.0; b[i] = y[i]; }
  lapack_dlarf1(m, v1, tau1, c);
  lapack_dlarf1(m, v1, tau1, b);
  int rank;
  double s0, s1, res = 0.0;
  if (m == 2) {
    /* path 1 (M < MNTHR): dgebrd directly; d = (beta1, c1), e = c0 */
    rank = lapack_dlalsd2(beta1, c[1], c[0], b[0], b[1], rcond, &s0, &s1);
  } else {
    /* path 1a: QR; H2 on c[1:] */
    double r12 = c[0];
    double alpha2 = c[1];
    double v2[LT_MAX_OBS];
    v2[0] = 1.0;
    for (int i = 2; i < m; i++) v2[i - 1] = c[i];
    double tau2 = lapack_dlarfg(m - 1, &alpha2, v2 + 1);
    double beta2 = alpha2;
    lapack_dlarf1(m - 1, v2, tau2, b + 1);
    rank = lapack_dlalsd2(beta1, beta2, r12, b[0], b[1], rcond, &s0, &s1);
    for (int k = 2; k < m; k++) res = res + b[k] * b[k];
  }
  if (rank < 0) return -1;
  *slope = s0;
  *icpt = s1;
  /* numpy returns residuals only when rank == n and m > n; np.sum([]) == 0.0 */
  *ssr = (rank == 2 && m > 2) ? res : 0.0;
  return rank == 2 ? 0 : -3;
}

/* ------------------------------------------------------------------------------------------ */
/* analyze (utils.py:735-789) on a compacted winner series                                      */
/* ------------------------------------------------------------------------------------------ */
int lto_analyze_series(int T, const int32_t* year, const double* val, double line_cost,
                       double* val_fit, double* fit_m, double* fit_b, double* right_m,
                       double* right_b, uint8_t* spike, uint8_t* vertex) {
  if (T <= 0) return LT_ST_EMPTY;
  if (T == 1) return LT_ST_SINGLE_YEAR;
  if (T > LT_MAX_YEARS) return LT_ST_NUMERIC;
  int status = LT_ST_OK;
  /* despike (utils.py:556-582): triples over the ORIGINAL series, first/last kept */
  uint8_t is_spike[LT_MAX_YEARS];
  double sd = lto_std(T, val);
  is_spike[0] = 0;
  double last_good = val[0];
  for (int i = 1; i < T - 1; i++) {
    double xv = val[i - 1], yv = val[i], zv = val[i + 1];
    int mono = (xv <= yv && yv <= zv) || (xv >= yv && yv >= zv);
    if (!mono && (fabs(yv - xv) > sd && fabs(yv - zv) > sd) && yv != last_good) {
      is_spike[i] = 1;
    } else {
      is_spike[i] = 0;
      last_good = yv;
    }
  }
  is_spike[T - 1] = 0;
  /* timeseries2int_series (utils.py:552-554): x = year - first year; dropna (utils.py:608) */
  double xs[LT_MAX_YEARS], ys[LT_MAX_YEARS];
  int pos[LT_MAX_YEARS]; /* position of the k-th non-spike point in the full series */
  int n = 0;
  for (int i = 0; i < T; i++) {
    if (is_spike[i]) continue;
    xs[n] = (double)(year[i] - year[0]);
    ys[n] = val[i];
    pos[n] = i;
    n++;
  }
  /* segmented_least_squares (utils.py:600-631): DP with first-minimum argmin */
  double OPT[LT_MAX_YEARS + 1]; /* OPT[j+1] = reference OPT[j]; OPT[0] = OPT[-1] = 0 */
  int arg[LT_MAX_YEARS];
  OPT[0] = 0.0;
  for (int j = 0; j < n; j++) {
    double best = 0.0;
    int bi = -1;
    for (int i = 0; i <= j; i++) {
      double e = 0.0;
      if (i != j) {
        double sm, sb, ssr;
        int rc = lto_lstsq(j - i + 1, xs + i, ys + i, &sm, &sb, &ssr);
        if (rc < 0) status |= LT_ST_NUMERIC;
        e = ssr;
      }
      double v = (e + line_cost) + OPT[i];
      if (bi < 0 || v < best) { best = v; bi = i; }
    }
    OPT[j + 1] = best;
    arg[j] = bi;
  }
  /* find_segments (utils.py:633-644): segment starts + last point */
  uint8_t is_v[LT_MAX_YEARS];
  memset(is_v, 0, sizeof(is_v));
  for (int j = n - 1; j >= 0; j = arg[j] - 1) is_v[arg[j]] = 1;
  is_v[n - 1] = 1;
  /* vertices2eqns (utils.py:646-669): LS over consecutive vertices (label-inclusive) */
  double em[LT_MAX_YEARS], eb[LT_MAX_YEARS]; /* eqn per non-spike point index (vertex only) */
  int vlist[LT_MAX_YEARS], nv = 0;
  for (int k = 0; k < n; k++) if (is_v[k]) vlist[nv++] = k;
  for (int q = 0; q + 1 < nv; q++) {
    int a = vlist[q], bnd = vlist[q + 1];
    double sm, sb, ssr;
    int rc = lto_lstsq(bnd - a + 1, xs + a, ys + a, &sm, &sb, &ssr);
    if (rc < 0) status |= LT_ST_NUMERIC;
    em[a] = sm;
    eb[a] = sb;
  }
  em[vlist[nv - 1]] = em[vlist[nv - 2]];
  eb[vlist[nv - 1]] = eb[vlist[nv - 2]];
  /* eqn_right per point of the full series (spikes included) */
  double rm[LT_MAX_YEARS], rb[LT_MAX_YEARS];
  uint8_t full_v[LT_MAX_YEARS];
  memset(full_v, 0, sizeof(full_v));
  for (int k = 0; k < n; k++) full_v[pos[k]] = is_v[k];
  {
    int k = 0;
    double cm = 0.0, cb = 0.0;
    for (int i = 0; i < T; i++) {
      if (!is_spike[i]) {
        if (is_v[k]) { cm = em[k]; cb = eb[k]; }
        k++;
      }
      rm[i] = cm;
      rb[i] = cb;
    }
  }
  /* eqns2fitted_points (utils.py:682-722) */
  for (int i = 0; i < T; i++) {
    double x = (double)(year[i] - year[0]);
    double fv, fm, fb;
    if (i == 0 || (rm[i - 1] == rm[i] && rb[i - 1] == rb[i])) {
      fv = (rm[i] * x) + rb[i];
      fm = rm[i]; fb = rb[i];
    } else {
      double fl = (rm[i - 1] * x) + rb[i - 1];
      double fr = (rm[i] * x) + rb[i];
      double raw = is_spike[i] ? NAN : val[i];
      if (fabs(fl - raw) <= fabs(fr - raw)) { fv = fl; fm = rm[i - 1]; fb = rb[i - 1]; }
      else { fv = fr; fm = rm[i]; fb = rb[i]; }
    }
    if (val_fit) val_fit[i] = fv;
    if (fit_m) fit_m[i] = fm;
    if (fit_b) fit_b[i] = fb;
    if (right_m) right_m[i] = rm[i];
    if (right_b) right_b[i] = rb[i];
    if (spike) spike[i] = is_spike[i];
    if (vertex) vertex[i] = full_v[i];
  }
  return status;
}

/* ------------------------------------------------------------------------------------------ */
/* change_labeling (utils.py:795-820) / Trendline.match_rule (classes.py:178-232)              */
/* ------------------------------------------------------------------------------------------ */
int lto_label(int T, const int32_t* year, const double* val_fit, const uint8_t* vertex,
              int n_rules, const lt_rule* rules, int pre_threshold_mode, uint8_t* matched,
              int32_t* onset_year, int32_t* duration, double* magnitude, double* initial_val) {
  int status = LT_ST_OK;
  for (int r = 0; r < n_rules; r++) {
    const lt_rule* R = &rules[r];
    int have = 0;
    int32_t w_on = 0, w_du = 0;
    double w_mag = 0.0, w_init = 0.0;
    int left = 0; /* parse_disturbances: first point is the left vertex (classes.py:163-164) */
    for (int p = 1; p < T; p++) {
      if (!vertex[p]) continue;
      int32_t on = year[left];
      int32_t du = year[p] - year[left];
      double init = val_fit[left];
      double mag = val_fit[left] - val_fit[p];
      left = p;
      int match = 1;
      if (R->onset_op == LT_Q_EQ && !((double)on == R->onset_val)) match = 0;
      else if (R->onset_op == LT_Q_LE && (double)on > R->onset_val) match = 0;
      else if (R->onset_op == LT_Q_GE && (double)on < R->onset_val) match = 0;
      if (R->duration_op == LT_Q_GT && (double)du <= R->duration_val) match = 0;
      else if (R->duration_op == LT_Q_LT && (double)du >= R->duration_val) match = 0;
      if (R->pre_op != LT_Q_UNSET) {
        if (pre_threshold_mode == LT_PRE_REFERENCE) {
          status |= LT_ST_PRE_THRESHOLD_ATTR; /* rule.threshold: AttributeError */
        } else if (R->pre_op == LT_Q_GT && init <= R->pre_val) match = 0;
        else if (R->pre_op == LT_Q_LT && init >= R->pre_val) match = 0;
      }
      if (!match) continue;
      int take = 0;
      if (!have) take = 1;
      else if (R->change_type == LT_CT_FD) take = on < w_on;
      else if (R->change_type == LT_CT_GD) take = mag > w_mag;
      else if (R->change_type == LT_CT_LD) take = du > w_du;
      if (take) { have = 1; w_on = on; w_du = du; w_mag = mag; w_init = init; }
    }
    if (matched) matched[r] = (uint8_t)have;
    if (onset_year) onset_year[r] = have ? w_on : LT_NODATA;
    if (duration) duration[r] = have ? w_du : LT_NODATA;
    if (magnitude) magnitude[r] = have ? w_mag : (double)LT_NODATA;
    if (initial_val) initial_val[r] = have ? w_init : (double)LT_NODATA;
  }
  return status;
}

/* ------------------------------------------------------------------------------------------ */
/* Tile driver: pick_winners (utils.py:491-521) + analyze + label per pixel, threaded.         */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  const lt_scene* scene;
  const lt_params* params;
  const lt_tile_in* in;
  const lt_tile_out* out;
  int64_t p0, p1;
} tile_job;

static void run_pixel(const lt_scene* S, const lt_params* P, const lt_tile_in* in,
                      const lt_tile_out* out, int64_t p) {
  const int Y = S->n_years;
  const int64_t is = in->stride, os = out->stride;
  int32_t year[LT_MAX_YEARS];
  double val[LT_MAX_YEARS];
  int slot_of[LT_MAX_YEARS];
  int T = 0, status = LT_ST_OK;
  for (int y = 0; y < Y; y++) {
    int best = -1, bd = 0;
    for (int k = S->slot_begin[y]; k < S->slot_begin[y + 1]; k++) {
      int o = S->order[k];
      if (in->obs_valid && !in->obs_valid[(int64_t)o * is + p]) continue;
      if (best < 0 || S->dist[k] < bd) { best = o; bd = S->dist[k]; }
    }
    if (out->winner) out->winner[(int64_t)y * os + p] = (int16_t)best;
    if (best >= 0) {
      if (S->feb29_bad && S->feb29_bad[y]) status |= LT_ST_FEB29;
      year[T] = S->year[y];
      val[T] = in->obs_val[(int64_t)best * is + p];
      slot_of[T] = y;
      T++;
    }
  }
  double vf[LT_MAX_YEARS], fm[LT_MAX_YEARS], fb[LT_MAX_YEARS], rm[LT_MAX_YEARS], rb[LT_MAX_YEARS];
  uint8_t sp[LT_MAX_YEARS], vx[LT_MAX_YEARS];
  int st = lto_analyze_series(T, year, val, P->line_cost, vf, fm, fb, rm, rb, sp, vx);
  status |= st;
  int ok = !(st & (LT_ST_EMPTY | LT_ST_SINGLE_YEAR));
  /* per-year outputs: absent years NaN / 0 */
  for (int y = 0, t = 0; y < Y; y++) {
    int present = (t < T && slot_of[t] == y);
    int64_t q = (int64_t)y * os + p;
    double nan = NAN;
    if (out->val_raw) out->val_raw[q] = present ? val[t] : nan;
    if (out->val_fit) out->val_fit[q] = (present && ok) ? vf[t] : nan;
    if (out->fit_m) out->fit_m[q] = (present && ok) ? fm[t] : nan;
    if (out->fit_b) out->fit_b[q] = (present && ok) ? fb[t] : nan;
    if (out->right_m) out->right_m[q] = (present && ok) ? rm[t] : nan;
    if (out->right_b) out->right_b[q] = (present && ok) ? rb[t] : nan;
    if (out->spike) out->spike[q] = (present && ok) ? sp[t] : 0;
    if (out->vertex) out->vertex[q] = (present && ok) ? vx[t] : 0;
    if (present) t++;
  }
  uint8_t mt[LT_MAX_RULES];
  int32_t on[LT_MAX_RULES], du[LT_MAX_RULES];
  double mg[LT_MAX_RULES], iv[LT_MAX_RULES];
  int R = P->n_rules;
  if (ok) {
    status |= lto_label(T, year, vf, vx, R, P->rules, P->pre_threshold_mode, mt, on, du, mg, iv);
  } else {
    for (int r = 0; r < R; r++) { mt[r] = 0; on[r] = du[r] = LT_NODATA; mg[r] = iv[r] = LT_NODATA; }
  }
  for (int r = 0; r < R; r++) {
    int64_t q = (int64_t)r * os + p;
    if (out->matched) out->matched[q] = mt[r];
    if (out->class_val) out->class_val[q] = mt[r] ? P->rules[r].class_val : LT_NODATA;
    if (out->onset_year) out->onset_year[q] = on[r];
    if (out->duration) out->duration[q] = du[r];
    if (out->magnitude) out->magnitude[q] = mg[r];
    if (out->initial_val) out->initial_val[q] = iv[r];
  }
  if (out->status) out->status[p] = status;
  if (out->n_years) out->n_years[p] = T;
}

static void* tile_worker(void* arg) {
  tile_job* J = (tile_job*)arg;
  for (int64_t p = J->p0; p < J->p1; p++) run_pixel(J->scene, J->params, J->in, J->out, p);
  return NULL;
}

int lto_analyze_tile(const lt_scene* scene, const lt_params* params, const lt_tile_in* in,
                     const lt_tile_out* out, int n_threads) {
  if (!scene || !params || !in || !out || !in->obs_val) return LT_ERR_ARG;
  if (scene->n_years > LT_MAX_YEARS || params->n_rules > LT_MAX_RULES) return LT_ERR_LIMIT;
  if (n_threads < 1) n_threads = 1;
  int64_t P = in->n_pix;
  if (n_threads > 256) n_threads = 256;
  pthread_t th[256];
  tile_job jobs[256];
  int64_t chunk = (P + n_threads - 1) / n_threads;
  int started = 0;
  for (int t = 0; t < n_threads; t++) {
    jobs[t].scene = scene; jobs[t].params = params; jobs[t].in = in; jobs[t].out = out;
    jobs[t].p0 = (int64_t)t * chunk;
    jobs[t].p1 = jobs[t].p0 + chunk < P ? jobs[t].p0 + chunk : P;
    if (jobs[t].p0 >= jobs[t].p1) break;
    if (n_threads == 1) { tile_worker(&jobs[t]); continue; }
    pthread_create(&th[t], NULL, tile_worker, &jobs[t]);
    started = t + 1;
  }
  for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
  return LT_OK;
}
