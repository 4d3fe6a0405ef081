// lt_lapack.h — np.linalg.lstsq([x | 1], y) for one segment, bit-for-bit as the reference reaches
// it (utils.py:594-597 → numpy 2.2.6 → OpenBLAS 0.3.29 SkylakeX dgelsd), restated for CDNA4.
//
// Arithmetic recipe: SURVEY.md Appendix A. Differences from a textbook Householder solve, all of
// which decide DP tie-breaks on integer Landsat data:
//   * dnrm2 is x87 code (80-bit accumulators, 64-bit significand): emulated here in integer
//     arithmetic (f80_* below) — the x87 unit has no counterpart on the GPU;
//   * dgemv_t sums in four interleaved lanes plus an FMA tail; daxpy/drot fuse (explicit fma());
//   * everything else is separately rounded binary64 (build with -ffp-contract=off).
// The segment vectors (the ones column after H1, b after H1/H2) are never materialised: every
// pass recomputes element k from x[k], y[k] and the pass-invariant scalars, so one lane carries a
// whole segment in ~20 registers. Functions are __host__ __device__ so the tests can run this exact
// code on the CPU against the oracle (tests/native/lapack_host_check.hip).
#pragma once
#ifndef __HIPCC_RTC__  // hiprtc (the JIT kernels, lt_jit.h) brings its own
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

namespace lt {

// ------------------------------------------------------------------------------------------------
// Non-negative soft float80: value = sig * 2^(exp - 63), sig normalised (bit 63 set) or 0.
// Only squares of doubles, sums of non-negatives and one final sqrt are ever needed (dnrm2).
// ------------------------------------------------------------------------------------------------
struct f80 {
  uint64_t sig;
  int32_t exp;
};

__host__ __device__ inline uint64_t dbl_bits(double d) { return __builtin_bit_cast(uint64_t, d); }

// x87 fmul of a double by itself: exact 106-bit product rounded to a 64-bit significand (RNE).
__host__ __device__ inline f80 f80_sq(double d) {
  uint64_t b = dbl_bits(d) & 0x7fffffffffffffffull;
  if (b == 0) return f80{0, 0};
  int32_t e = (int32_t)(b >> 52);
  uint64_t m = b & 0x000fffffffffffffull;
  if (e == 0) {  // subnormal: normalise
    int sh = __builtin_clzll(m) - 11;
    m <<= sh;
    e = 1 - sh;
  } else {
    m |= 0x0010000000000000ull;
  }
  unsigned __int128 P = (unsigned __int128)m * m;  // in [2^104, 2^106)
  int sh = ((uint64_t)(P >> 64) >> 41) ? 42 : 41;
  uint64_t sig = (uint64_t)(P >> sh);
  uint64_t rem = (uint64_t)P & ((1ull << sh) - 1);
  uint64_t half = 1ull << (sh - 1);
  int32_t ex = sh + 2 * e - 2087;
  if (rem > half || (rem == half && (sig & 1))) {
    sig++;
    if (sig == 0) {
      sig = 1ull << 63;
      ex++;
    }
  }
  return f80{sig, ex};
}

// x87 fadd of two non-negative extended values, RNE to a 64-bit significand.
__host__ __device__ inline f80 f80_add(f80 a, f80 b) {
  if (b.sig == 0) return a;
  if (a.sig == 0) return b;
  if (a.exp < b.exp) {
    f80 t = a;
    a = b;
    b = t;
  }
  int32_t d = a.exp - b.exp;
  if (d > 64) return a;  // b < half an ulp of a
  uint64_t bhi, blo;
  if (d == 0) {
    bhi = b.sig;
    blo = 0;
  } else if (d < 64) {
    bhi = b.sig >> d;
    blo = b.sig << (64 - d);
  } else {
    bhi = 0;
    blo = b.sig;
  }
  uint64_t hi = a.sig + bhi;
  uint64_t sig, rbit, sticky;
  int32_t ex = a.exp;
  if (hi < a.sig) {  // carry out: 65-bit sum
    sig = (1ull << 63) | (hi >> 1);
    rbit = hi & 1;
    sticky = blo != 0;
    ex++;
  } else {
    sig = hi;
    rbit = blo >> 63;
    sticky = (blo << 1) != 0;
  }
  if (rbit && (sticky || (sig & 1))) {
    sig++;
    if (sig == 0) {
      sig = 1ull << 63;
      ex++;
    }
  }
  return f80{sig, ex};
}

// (double) sqrtl(t): square root rounded to 64 bits (RNE), then to 53 bits (RNE) — the double
// rounding of x87 fsqrt followed by fstpl.
__host__ __device__ inline double f80_sqrt_to_double(f80 t) {
  if (t.sig == 0) return 0.0;
  int32_t ep = t.exp - 63;           // t = sig * 2^ep
  int s = ((ep - 63) & 1) ? 64 : 63;  // ep - s even
  unsigned __int128 N = (unsigned __int128)t.sig << s;  // in [2^126, 2^128)
  int32_t half_e = (ep - s) / 2;      // exact (even)
  // integer square root: floating estimate, one Newton correction, exact fix-up
  double Nd = (double)(uint64_t)(N >> 64) * 0x1p64 + (double)(uint64_t)N;
  double qd = __builtin_sqrt(Nd);
  uint64_t q = qd >= 0x1p64 ? ~0ull : (uint64_t)qd;
  {
    unsigned __int128 q2 = (unsigned __int128)q * q;
    double diff = q2 > N ? -(double)(q2 - N) : (double)(N - q2);
    double dq = diff / (2.0 * (double)q);
    int64_t step = (int64_t)(dq >= 0 ? dq + 0.5 : dq - 0.5);
    q = (uint64_t)((int64_t)q + step);
  }
  while ((unsigned __int128)q * q > N) q--;
  while (q != ~0ull && (unsigned __int128)(q + 1) * (q + 1) <= N) q++;
  unsigned __int128 rem = N - (unsigned __int128)q * q;
  int32_t ex = half_e;
  if (rem > (unsigned __int128)q) {  // sqrt(N) > q + 1/2 (never exactly)
    if (q == ~0ull) {
      q = 1ull << 63;
      ex++;
    } else {
      q++;
    }
  }
  // round the 64-bit significand to 53 bits
  uint64_t mant = q >> 11;
  uint64_t r = q & 0x7ff;
  if (r > 0x400 || (r == 0x400 && (mant & 1))) {
    mant++;
    if (mant == (1ull << 53)) {
      mant = 1ull << 52;
      ex++;
    }
  }
  return __builtin_ldexp((double)mant, ex + 11);
}

// ------------------------------------------------------------------------------------------------
// Streaming BLAS pieces. Element k of the vector is produced by a callable `get(k)`.
// ------------------------------------------------------------------------------------------------

// OpenBLAS dnrm2_k SkylakeX over n elements: 4 x87 accumulators in 8-element blocks.
template <class G>
__host__ __device__ inline double nrm2(int n, G get) {
  if (n <= 0) return 0.0;
  if (n == 1) return __builtin_fabs(get(0));
  f80 a0{0, 0}, a1{0, 0}, a2{0, 0}, a3{0, 0};
  int n8 = n & ~7, j = 0;
  for (; j < n8; j += 4) {
    a0 = f80_add(a0, f80_sq(get(j)));
    a1 = f80_add(a1, f80_sq(get(j + 1)));
    a2 = f80_add(a2, f80_sq(get(j + 2)));
    a3 = f80_add(a3, f80_sq(get(j + 3)));
  }
  for (; j < n; j++) a0 = f80_add(a0, f80_sq(get(j)));
  f80 t = f80_add(f80_add(f80_add(a0, a2), a1), a3);
  return f80_sqrt_to_double(t);
}

// ------------------------------------------------------------------------------------------------
// The same dnrm2 in binary64 pairs (the GPU's fp64 pipes instead of 64-bit integer emulation).
// An extended value V is held as xdd{hi, lo}: V = hi + lo exactly, |lo| <= ulp53(hi) / 2, and V
// has a 64-bit significand (lo is a multiple of ulp64(V)). Each x87 operation becomes an
// error-free transformation (exact product / exact sum as a pair) followed by rounding the low
// part to a multiple of ulp64(V) with round-half-even: (lo + C) - C with ulp(C) = ulp64(V). Since
// hi is a multiple of 2^11 ulp64(V), the parity of the rounded low part is the parity of V's
// 64-bit significand, so ties go the x87 way.
// The sum is exact while the two exponents differ by <= 38 and the squares stay inside
// [2^-900, 2^1000]; outside that `slow` is raised and the caller redoes the norm with nrm2().
// ------------------------------------------------------------------------------------------------
struct xdd {
  double hi, lo;
};

// E with 2^E <= hi + lo < 2^(E+1) (hi > 0)
__host__ __device__ inline int xdd_exp(double hi, double lo) {
  int e;
  const double mt = __builtin_frexp(hi, &e);  // hi = mt * 2^e, mt in [0.5, 1)
  return (mt == 0.5 && lo < 0.0) ? e - 2 : e - 1;
}

// hi = RN(hi + lo), |lo| <= ulp53(hi) / 2: round hi + lo to a 64-bit significand (RNE)
__host__ __device__ inline xdd xdd_round64(double hi, double lo) {
  const double C = __builtin_ldexp(1.5, xdd_exp(hi, lo) - 11);  // ulp(C) = ulp64(hi + lo)
  return xdd{hi, (lo + C) - C};
}

// x87 fmul of a double by itself
__host__ __device__ inline xdd xdd_sq(double c, bool& slow) {
  const double p = c * c;
  const double e = __builtin_fma(c, c, -p);  // exact: c^2 = p + e
  const double a = __builtin_fabs(c);
  slow |= (a != 0.0 && a < 0x1p-450) || a > 0x1p500;
  return xdd_round64(p, e);
}

// x87 fadd of two non-negative extended values
__host__ __device__ inline xdd xdd_add(xdd A, xdd B, bool& slow) {
  int ea, eb;
  __builtin_frexp(A.hi, &ea);
  __builtin_frexp(B.hi, &eb);
  slow |= A.hi != 0.0 && B.hi != 0.0 && (ea - eb > 38 || eb - ea > 38);
  const double s = A.hi + B.hi;  // TwoSum: A.hi + B.hi = s + t
  const double bb = s - A.hi;
  const double t = (A.hi - (s - bb)) + (B.hi - bb);
  const double r = (t + A.lo) + B.lo;  // exact: all three are multiples of ulp64 of the smaller
  const double s2 = s + r;             // TwoSum: s + r = s2 + r2
  const double b2 = s2 - s;
  const double r2 = (s - (s2 - b2)) + (r - b2);
  return xdd_round64(s2, r2);
}

__host__ __device__ inline f80 xdd_to_f80(xdd v) {
  if (v.hi == 0.0) return f80{0, 0};
  const int E = xdd_exp(v.hi, v.lo);
  // hi * 2^(63-E) is an integer in [2^63, 2^64]: scale by 2^(62-E), double in integers (2^64
  // wraps to 0 and the negative low part brings it back)
  const uint64_t h = (uint64_t)__builtin_ldexp(v.hi, 62 - E) << 1;
  const int64_t l = (int64_t)__builtin_ldexp(v.lo, 63 - E);
  return f80{h + (uint64_t)l, E};
}

// (double) sqrtl(V) — x87 fsqrt (RN to 64 bits) then the store to binary64 (RN to 53 bits) — for
// V = hi + lo as above, in binary64: s = sqrt(hi), d ~ (V - s^2) / 2s from the exact remainder,
// so sqrt(V) = s + d to ~2^-100 relative. The 64-bit rounding is k = round(d / ulp64) (sqrt(V)
// is never a 64-bit midpoint; within 2^-20 ulp64 of one `slow` is raised), the 53-bit rounding of
// s + k ulp64 is integer work on k. s a power of two with d < 0 (a binade edge) raises `slow`.
__host__ __device__ inline double xdd_sqrt_to_double(double hi, double lo, bool& slow) {
  if (hi == 0.0) return 0.0;
  const double s = __builtin_sqrt(hi);
  const double e1 = __builtin_fma(-s, s, hi);  // hi - s^2, exact for a correctly rounded s
  const double d = (e1 + lo) / (2.0 * s);
  int E;
  const double mt = __builtin_frexp(s, &E);  // s in [2^(E-1), 2^E): ulp53 = 2^(E-53)
  const double kd = __builtin_ldexp(d, 64 - E);  // d in units of ulp64 = 2^(E-64)
  const double kf = __builtin_floor(kd);
  slow |= (mt == 0.5 && d < 0.0) || __builtin_fabs(kd - kf - 0.5) < 0x1p-20 ||
          __builtin_fabs(kd) > 0x1p13;
  const int k = (int)kf + (kd - kf > 0.5 ? 1 : 0);  // RN(sqrt V) to 64 bits = s + k ulp64
  int a = k >> 11;                                  // s + a ulp53 <= q64 < s + (a+1) ulp53
  const int b = k - (a << 11);
  const int odd = (int)((dbl_bits(s) + (uint64_t)(int64_t)a) & 1);
  if (b > 1024 || (b == 1024 && odd)) a++;
  return s + __builtin_ldexp((double)a, E - 53);
}

// nrm2 (OpenBLAS dnrm2_k SkylakeX) on xdd accumulators; identical result unless `slow` is raised
template <class G>
__host__ __device__ inline double nrm2_dd(int n, G get, bool& slow) {
  if (n <= 0) return 0.0;
  if (n == 1) return __builtin_fabs(get(0));
  xdd a0{0.0, 0.0}, a1{0.0, 0.0}, a2{0.0, 0.0}, a3{0.0, 0.0};
  int n8 = n & ~7, j = 0;
  for (; j < n8; j += 4) {
    a0 = xdd_add(a0, xdd_sq(get(j), slow), slow);
    a1 = xdd_add(a1, xdd_sq(get(j + 1), slow), slow);
    a2 = xdd_add(a2, xdd_sq(get(j + 2), slow), slow);
    a3 = xdd_add(a3, xdd_sq(get(j + 3), slow), slow);
  }
  for (; j < n; j++) a0 = xdd_add(a0, xdd_sq(get(j), slow), slow);
  const xdd t = xdd_add(xdd_add(xdd_add(a0, a2, slow), a1, slow), a3, slow);
  return xdd_sqrt_to_double(t.hi, t.lo, slow);
}

// OpenBLAS dgemv_t SkylakeX, one column: sum_k a(k) v(k) with 4 interleaved lanes + FMA tail.
template <class GA, class GV>
__host__ __device__ inline double gemv_t1(int m, GA a, GV v) {
  int m3 = m & 3, m1 = m - m3;
  double y = 0.0;
  if (m1 > 0) {
    double L0 = 0.0, L1 = 0.0, L2 = 0.0, L3 = 0.0;
    for (int i = 0; i < m1; i += 4) {
      L0 = L0 + a(i) * v(i);
      L1 = L1 + a(i + 1) * v(i + 1);
      L2 = L2 + a(i + 2) * v(i + 2);
      L3 = L3 + a(i + 3) * v(i + 3);
    }
    double r = (L0 + L2) + (L1 + L3);
    y = __builtin_fma(r, 1.0, y);
  }
  if (m3 == 1) {
    y = __builtin_fma(a(m1), v(m1), y);
  } else if (m3 == 2) {
    y = y + __builtin_fma(a(m1), v(m1), a(m1 + 1) * v(m1 + 1));
  } else if (m3 == 3) {
    y = y + __builtin_fma(a(m1 + 2), v(m1 + 2), __builtin_fma(a(m1), v(m1), a(m1 + 1) * v(m1 + 1)));
  }
  return y;
}

__host__ __device__ inline double dlapy2(double x, double y) {
  double xa = __builtin_fabs(x), ya = __builtin_fabs(y);
  double w = xa > ya ? xa : ya;
  double z = xa < ya ? xa : ya;
  if (z == 0.0) return w;
  double t = z / w;
  return w * __builtin_sqrt(1.0 + t * t);
}

__host__ __device__ inline double fsign(double a, double b) {
  return __builtin_copysign(__builtin_fabs(a), b);
}

// DLASV2 (LAPACK 3.x), literal transcription.
__host__ __device__ inline void dlasv2(double f, double g, double h, double& ssmin, double& ssmax,
                                       double& snr, double& csr, double& snl, double& csl) {
  const double eps = 0x1p-53;
  double ft = f, fa = __builtin_fabs(ft), ht = h, ha = __builtin_fabs(h);
  int pmax = 1;
  bool swap = ha > fa;
  if (swap) {
    pmax = 3;
    double tmp = ft;
    ft = ht;
    ht = tmp;
    tmp = fa;
    fa = ha;
    ha = tmp;
  }
  double gt = g, ga = __builtin_fabs(gt);
  double clt, crt, slt, srt, smin, smax;
  if (ga == 0.0) {
    smin = ha;
    smax = fa;
    clt = 1.0;
    crt = 1.0;
    slt = 0.0;
    srt = 0.0;
  } else {
    bool gasmal = true;
    if (ga > fa) {
      pmax = 2;
      if ((fa / ga) < eps) {
        gasmal = false;
        smax = ga;
        smin = (ha > 1.0) ? fa / (ga / ha) : (fa / ga) * ha;
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
      double s = __builtin_sqrt(tt + mm);
      double r = (l == 0.0) ? __builtin_fabs(m) : __builtin_sqrt(l * l + mm);
      double a = 0.5 * (s + r);
      smin = ha / a;
      smax = fa * a;
      if (mm == 0.0) {
        if (l == 0.0) t = fsign(2.0, ft) * fsign(1.0, gt);
        else t = gt / fsign(d, ft) + m / t;
      } else {
        t = (m / (s + t) + m / (r + l)) * (1.0 + a);
      }
      l = __builtin_sqrt(t * t + 4.0);
      crt = 2.0 / l;
      srt = t / l;
      clt = (crt + srt * m) / a;
      slt = ((ht / ft) * srt) / a;
    }
  }
  if (swap) {
    csl = srt; snl = crt; csr = slt; snr = clt;
  } else {
    csl = clt; snl = slt; csr = crt; snr = srt;
  }
  double tsign;
  if (pmax == 1) tsign = fsign(1.0, csr) * fsign(1.0, csl) * fsign(1.0, f);
  else if (pmax == 2) tsign = fsign(1.0, snr) * fsign(1.0, csl) * fsign(1.0, g);
  else tsign = fsign(1.0, snr) * fsign(1.0, snl) * fsign(1.0, h);
  ssmax = fsign(smax, tsign);
  ssmin = fsign(smin, tsign * fsign(1.0, f) * fsign(1.0, h));
}

// DLALSD, N = 2: DLASDQ/DBDSQR on the 2x2 upper bidiagonal (d1, e; d2), solve, back-transform.
// Split in the part that depends on R = (d1, e; d2) only (dlalsd2_r: scaling, DLASV2 rotation,
// sign fixes, the ascending re-sort, rank) and the part applied to b (dlalsd2_b), so a segment's
// x-only factorisation can be computed once and reused (lsq_factor / lsq_apply below).
struct lalsd2_r {
  double mul, csl, snl, vt00, vt01, vt10, vt11, inv1, inv2;
  int32_t rank;  // numerical rank 0..2, or -1 for the DLASCL rescaling path (not emulated)
  uint8_t rot, swap, r1, r2;
  uint8_t zero;  // org == 0: zero solution
  uint8_t pad[3];
};

__host__ __device__ inline lalsd2_r dlalsd2_r(double d1, double d2, double e, double rcond) {
  lalsd2_r R{};
  const double eps = 0x1p-53, unfl = 0x1p-1022;
  const double tolmul = 98.70149282610821;  // max(10, min(100, eps^(-1/8)))
  double rcnd = (rcond > 0.0 && rcond < 1.0) ? rcond : eps;
  double org = __builtin_fabs(d1);
  if (__builtin_fabs(d2) > org) org = __builtin_fabs(d2);
  if (__builtin_fabs(e) > org) org = __builtin_fabs(e);
  if (org == 0.0) {
    R.zero = 1;
    R.rank = 0;
    return R;
  }
  if (!(org > 0x1p-900 && org < 0x1p900)) {
    R.rank = -1;
    return R;
  }
  const double mul = 1.0 / org;
  d1 *= mul;
  d2 *= mul;
  e *= mul;
  double vt00 = 1.0, vt01 = 0.0, vt10 = 0.0, vt11 = 1.0;
  double sminoa = __builtin_fabs(d1);
  if (sminoa != 0.0) {
    double mu = __builtin_fabs(d2) * (sminoa / (sminoa + __builtin_fabs(e)));
    if (mu < sminoa) sminoa = mu;
  }
  sminoa = sminoa / __builtin_sqrt(2.0);
  double thresh = (tolmul * eps) * sminoa;
  const double floor_ = 6.0 * (2.0 * (2.0 * unfl));
  if (floor_ > thresh) thresh = floor_;
  if (__builtin_fabs(e) > thresh) {
    double ssmin, ssmax, snr, csr, snl, csl;
    dlasv2(d1, e, d2, ssmin, ssmax, snr, csr, snl, csl);
    d1 = ssmax;
    d2 = ssmin;
    double a0 = vt00, c0 = vt10;
    vt00 = __builtin_fma(csr, a0, snr * c0);
    vt10 = __builtin_fma(csr, c0, -(snr * a0));
    double a1 = vt01, c1 = vt11;
    vt01 = __builtin_fma(csr, a1, snr * c1);
    vt11 = __builtin_fma(csr, c1, -(snr * a1));
    R.rot = 1;
    R.csl = csl;
    R.snl = snl;
  }
  if (d1 < 0.0) {
    d1 = -d1;
    vt00 = -vt00;
    vt01 = -vt01;
  }
  if (d2 < 0.0) {
    d2 = -d2;
    vt10 = -vt10;
    vt11 = -vt11;
  }
  // DBDSQR leaves them descending, DLASDQ re-sorts ascending: net, one swap iff d1 > d2
  if (d1 > d2) {
    double t = d1; d1 = d2; d2 = t;
    t = vt00; vt00 = vt10; vt10 = t;
    t = vt01; vt01 = vt11; vt11 = t;
    R.swap = 1;
  }
  const double dmax = __builtin_fabs(d1) > __builtin_fabs(d2) ? __builtin_fabs(d1) : __builtin_fabs(d2);
  const double tol2 = rcnd * dmax;
  R.rank = 0;
  if (!(d1 <= tol2)) {
    R.inv1 = 1.0 / d1;
    R.r1 = 1;
    R.rank++;
  }
  if (!(d2 <= tol2)) {
    R.inv2 = 1.0 / d2;
    R.r2 = 1;
    R.rank++;
  }
  R.mul = mul;
  R.vt00 = vt00;
  R.vt01 = vt01;
  R.vt10 = vt10;
  R.vt11 = vt11;
  return R;
}

__host__ __device__ inline void dlalsd2_b(const lalsd2_r& R, double b1, double b2, double& x0,
                                          double& x1) {
  if (R.zero) {
    x0 = 0.0;
    x1 = 0.0;
    return;
  }
  if (R.rot) {
    const double p = b1, q = b2;
    b1 = __builtin_fma(R.csl, p, R.snl * q);
    b2 = __builtin_fma(R.csl, q, -(R.snl * p));
  }
  if (R.swap) {
    const double t = b1;
    b1 = b2;
    b2 = t;
  }
  b1 = R.r1 ? b1 * R.inv1 : 0.0;
  b2 = R.r2 ? b2 * R.inv2 : 0.0;
  const double s0 = __builtin_fma(R.vt10, b2, R.vt00 * b1);
  const double s1 = __builtin_fma(R.vt11, b2, R.vt01 * b1);
  x0 = s0 * R.mul;
  x1 = s1 * R.mul;
}

// Returns the numerical rank, or -1 for the DLASCL rescaling path (not emulated).
__host__ __device__ inline int dlalsd2(double d1, double d2, double e, double b1, double b2,
                                       double rcond, double& x0, double& x1) {
  const lalsd2_r R = dlalsd2_r(d1, d2, e, rcond);
  if (R.rank < 0) return -1;
  dlalsd2_b(R, b1, b2, x0, x1);
  return R.rank;
}

// ------------------------------------------------------------------------------------------------
// least_squares (utils.py:584-598) of one segment of m >= 2 points given by X(k), Y(k).
// want_solution = false skips DLALSD (the DP needs only the residual; numpy still reports
// residuals only at rank 2, which the segment's distinct x guarantee — checked by the caller via
// lstsq_rank_ok when needed). Returns 0 on success, < 0 for paths not emulated.
// ------------------------------------------------------------------------------------------------
template <class GX, class GY>
__host__ __device__ inline int lstsq_segment(int m, GX X, GY Y, bool want_solution, double& slope,
                                             double& icpt, double& ssr) {
  const double rcond = 0x1p-52 * (double)(m > 2 ? m : 2);
  // DGELSD: B == 0 gives the zero solution at rank 0 (numpy then reports no residuals → 0.0);
  // B or A outside [SMLNUM, BIGNUM] = [2^-970, 2^970] would be rescaled (not emulated).
  {
    double bnrm = 0.0, anrm = 1.0;
    for (int k = 0; k < m; k++) {
      bnrm = __builtin_fmax(bnrm, __builtin_fabs(Y(k)));
      anrm = __builtin_fmax(anrm, __builtin_fabs(X(k)));
    }
    if (bnrm == 0.0) {
      slope = 0.0;
      icpt = 0.0;
      ssr = 0.0;
      return 0;
    }
    if (bnrm < 0x1p-970 || bnrm > 0x1p970 || anrm > 0x1p970) return -1;
  }
  // H1 = DLARFG(m, x0, x[1:])
  double alpha = X(0);
  double xn = nrm2(m - 1, [&](int k) { return X(k + 1); });
  double tau1 = 0.0, beta1 = alpha, s1 = 0.0;
  if (xn != 0.0) {
    beta1 = -__builtin_copysign(dlapy2(alpha, xn), alpha);
    tau1 = (beta1 - alpha) / beta1;
    s1 = 1.0 / (alpha - beta1);
  }
  auto v1 = [&](int k) { return k == 0 ? 1.0 : X(k) * s1; };
  // DLARF(v1, tau1) on the ones column and on y
  int lastv = m;
  double sc = 0.0, sb = 0.0;
  bool c_upd = false, b_upd = false;
  if (tau1 != 0.0) {
    while (lastv > 1 && v1(lastv - 1) == 0.0) lastv--;
    double w = gemv_t1(lastv, [](int) { return 1.0; }, v1);
    sc = (-tau1) * w;
    c_upd = true;
    bool any = false;
    for (int k = 0; k < lastv && !any; k++) any = Y(k) != 0.0;
    if (any) {
      double wb = gemv_t1(lastv, Y, v1);
      sb = (-tau1) * wb;
      b_upd = true;
    }
  }
  auto C = [&](int k) { return (c_upd && k < lastv) ? __builtin_fma(sc, v1(k), 1.0) : 1.0; };
  auto B = [&](int k) { return (b_upd && k < lastv) ? __builtin_fma(sb, v1(k), Y(k)) : Y(k); };
  int rank;
  double s0 = 0.0, sI = 0.0, res = 0.0;
  if (m == 2) {
    slope = 0.0;
    icpt = 0.0;
    ssr = 0.0;
    if (!want_solution) return 0;
    rank = dlalsd2(beta1, C(1), C(0), B(0), B(1), rcond, s0, sI);
  } else {
    double r12 = C(0);
    double alpha2 = C(1);
    double xn2 = nrm2(m - 2, [&](int k) { return C(k + 2); });
    double tau2 = 0.0, beta2 = alpha2, s2 = 0.0;
    if (xn2 != 0.0) {
      beta2 = -__builtin_copysign(dlapy2(alpha2, xn2), alpha2);
      tau2 = (beta2 - alpha2) / beta2;
      s2 = 1.0 / (alpha2 - beta2);
    }
    // v2 over b[1:]: v2(0) = 1, v2(k) = c(k+1) * s2
    auto v2 = [&](int k) { return k == 0 ? 1.0 : C(k + 1) * s2; };
    int lastv2 = m - 1;
    double sb2 = 0.0;
    bool b2_upd = false;
    if (tau2 != 0.0) {
      while (lastv2 > 1 && v2(lastv2 - 1) == 0.0) lastv2--;
      bool any = false;
      for (int k = 0; k < lastv2 && !any; k++) any = B(k + 1) != 0.0;
      if (any) {
        double w2 = gemv_t1(lastv2, [&](int k) { return B(k + 1); }, v2);
        sb2 = (-tau2) * w2;
        b2_upd = true;
      }
    }
    auto B2 = [&](int k) {  // final b (k >= 1)
      double bk = B(k);
      return (b2_upd && k - 1 < lastv2) ? __builtin_fma(sb2, v2(k - 1), bk) : bk;
    };
    for (int k = 2; k < m; k++) {
      double bk = B2(k);
      res = res + bk * bk;
    }
    if (!want_solution) {
      slope = 0.0;
      icpt = 0.0;
      ssr = res;
      return 0;
    }
    rank = dlalsd2(beta1, beta2, r12, B(0), B2(1), rcond, s0, sI);
  }
  if (rank < 0) return -1;
  slope = s0;
  icpt = sI;
  ssr = (rank == 2 && m > 2) ? res : 0.0;
  return rank == 2 ? 0 : -3;
}

// ------------------------------------------------------------------------------------------------
// The same least_squares for integer x (year offsets 0..255, the only x the analysis produces),
// with the passes fused: bit-identical to lstsq_segment (tests/test_lapack_emulation.py).
//   * dnrm2(x[1:]) is an exact integer sum of squares (the x87 accumulators never round below
//     2^64), so only its sqrt needs the soft-float80 path;
//   * both dgemv_t of H1 (ones . v1 and y . v1) share one pass, with DGELSD's B == 0 test and
//     DLARF's nonzero scan folded in;
//   * the residual pass runs only when need_ssr.
// x strictly increasing (so v1[k] != 0 for k >= 1) is required and checked (rc -4 otherwise).
// ------------------------------------------------------------------------------------------------
__host__ __device__ inline f80 f80_from_u64(uint64_t s) {
  if (s == 0) return f80{0, 0};
  const int lz = __builtin_clzll(s);
  return f80{s << lz, 63 - lz};  // value = sig * 2^(exp - 63) = s
}

// The x-only half of lstsq_xint: everything that depends on the segment's x values alone (the
// H1 reflector and the ones column it produces, H2 and its trimmed length, DLALSD's R part).
// Segments with the same x values share it, so the analysis keeps a device table of the common
// x-sets (lt_abi.hip) and applies only the y half per pixel. Identical operations in the same
// order as one fused lstsq: lstsq_xint(m, X, Y) == lsq_apply(lsq_factor(m, X), X, Y) bit for bit.
struct lsq_xf {
  double s1, ntau1, sc;  // v1(k) = x_k * s1 (k >= 1); sb = ntau1 * (y . v1); C(k) = fma(sc, v1(k), 1)
  double s2, ntau2;      // m >= 3: v2(k) = C(k+1) * s2 (k >= 1); sb2 = ntau2 * (b[1:] . v2)
  lalsd2_r R;            // DLALSD on R = (beta1, r12; beta2)
  int16_t m, lastv2;
  int8_t rc;             // 0, or -4 (x not strictly increasing)
  uint8_t tau2nz;
  uint8_t pad[2];
};

template <class GX>
__host__ __device__ inline void lsq_factor(int m, GX X, lsq_xf& f) {
  f = lsq_xf{};
  f.m = (int16_t)m;
  const double rcond = 0x1p-52 * (double)(m > 2 ? m : 2);
  // H1: alpha = x0, ||x[1:]|| from the exact integer sum of squares
  const int x0 = X(0);
  uint64_t S = 0;
  int xprev = x0;
  for (int k = 1; k < m; k++) {
    const int xk = X(k);
    if (xk <= xprev) {
      f.rc = -4;
      return;
    }
    xprev = xk;
    S += (uint64_t)((int64_t)xk * xk);
  }
  const double alpha = (double)x0;
  double xn = (double)X(1);
  if (m > 2) {
    bool slow = S >= (1ull << 53);
    xn = xdd_sqrt_to_double((double)S, 0.0, slow);
    if (slow) xn = f80_sqrt_to_double(f80_from_u64(S));
  }
  const double beta1 = -__builtin_copysign(dlapy2(alpha, xn), alpha);  // xn > 0
  const double tau1 = (beta1 - alpha) / beta1;
  const double s1 = 1.0 / (alpha - beta1);
  // pass A, ones half: gemv_t(ones, v1) (4 interleaved lanes + FMA tail)
  const int m3 = m & 3, m1 = m - m3;
  double A0 = 0.0, A1 = 0.0, A2 = 0.0, A3 = 0.0;
  for (int i = 0; i < m1; i += 4) {
    A0 = A0 + (i == 0 ? 1.0 : (double)X(i) * s1);
    A1 = A1 + (double)X(i + 1) * s1;
    A2 = A2 + (double)X(i + 2) * s1;
    A3 = A3 + (double)X(i + 3) * s1;
  }
  double wo = 0.0;
  if (m1 > 0) wo = __builtin_fma((A0 + A2) + (A1 + A3), 1.0, 0.0);
  auto v1 = [&](int k) { return k == 0 ? 1.0 : (double)X(k) * s1; };
  if (m3 == 1) {
    wo = __builtin_fma(1.0, v1(m1), wo);
  } else if (m3 == 2) {
    wo = wo + __builtin_fma(1.0, v1(m1), 1.0 * v1(m1 + 1));
  } else if (m3 == 3) {
    wo = wo + __builtin_fma(1.0, v1(m1 + 2), __builtin_fma(1.0, v1(m1), 1.0 * v1(m1 + 1)));
  }
  const double sc = (-tau1) * wo;
  auto C = [&](int k) { return __builtin_fma(sc, v1(k), 1.0); };
  f.s1 = s1;
  f.ntau1 = -tau1;
  f.sc = sc;
  if (m == 2) {
    f.R = dlalsd2_r(beta1, C(1), C(0), rcond);
    return;
  }
  // pass B: H2 on c[1:], ||c[2:]|| in binary64 pairs (soft-float80 on the rare fallback)
  const double r12 = C(0), alpha2 = C(1);
  bool slow = false;
  double xn2 = nrm2_dd(m - 2, [&](int k) { return C(k + 2); }, slow);
  if (slow) xn2 = nrm2(m - 2, [&](int k) { return C(k + 2); });
  double tau2 = 0.0, beta2 = alpha2, s2 = 0.0;
  if (xn2 != 0.0) {
    beta2 = -__builtin_copysign(dlapy2(alpha2, xn2), alpha2);
    tau2 = (beta2 - alpha2) / beta2;
    s2 = 1.0 / (alpha2 - beta2);
  }
  int lastv2 = m - 1;
  if (tau2 != 0.0) {
    auto v2 = [&](int k) { return k == 0 ? 1.0 : C(k + 1) * s2; };
    while (lastv2 > 1 && v2(lastv2 - 1) == 0.0) lastv2--;
  }
  f.s2 = s2;
  f.ntau2 = -tau2;
  f.tau2nz = tau2 != 0.0;
  f.lastv2 = (int16_t)lastv2;
  f.R = dlalsd2_r(beta1, beta2, r12, rcond);
}

// The y half: DGELSD's B == 0 shortcut and range check, H1 and H2 applied to y, the residual
// (need_ssr) and the solve (need_solution). X must give the x values f was factored from.
template <class GX, class GY>
__host__ __device__ inline int lsq_apply(const lsq_xf& f, GX X, GY Y, bool need_solution,
                                         bool need_ssr, double& slope, double& icpt, double& ssr) {
  slope = 0.0;
  icpt = 0.0;
  ssr = 0.0;
  if (f.rc < 0) return f.rc;
  const int m = f.m;
  const double s1 = f.s1;
  auto v1 = [&](int k) { return k == 0 ? 1.0 : (double)X(k) * s1; };
  // pass A, y half: gemv_t(y, v1) (4 interleaved lanes + FMA tail), B == 0 test
  const int m3 = m & 3, m1 = m - m3;
  double Q0 = 0.0, Q1 = 0.0, Q2 = 0.0, Q3 = 0.0;
  double bmax = 0.0;
  for (int i = 0; i < m1; i += 4) {
    const double y0 = Y(i), ya = Y(i + 1), yb = Y(i + 2), yc = Y(i + 3);
    Q0 = Q0 + y0 * v1(i);
    Q1 = Q1 + ya * v1(i + 1);
    Q2 = Q2 + yb * v1(i + 2);
    Q3 = Q3 + yc * v1(i + 3);
    bmax = __builtin_fmax(bmax, __builtin_fmax(__builtin_fmax(__builtin_fabs(y0),
                                                              __builtin_fabs(ya)),
                                               __builtin_fmax(__builtin_fabs(yb),
                                                              __builtin_fabs(yc))));
  }
  double wy = 0.0;
  if (m1 > 0) wy = __builtin_fma((Q0 + Q2) + (Q1 + Q3), 1.0, 0.0);
  if (m3 > 0) {
    const double ta = v1(m1), ya = Y(m1);
    bmax = __builtin_fmax(bmax, __builtin_fabs(ya));
    if (m3 == 1) {
      wy = __builtin_fma(ya, ta, wy);
    } else {
      const double tb = v1(m1 + 1), yb = Y(m1 + 1);
      bmax = __builtin_fmax(bmax, __builtin_fabs(yb));
      if (m3 == 2) {
        wy = wy + __builtin_fma(ya, ta, yb * tb);
      } else {
        const double tc = v1(m1 + 2), yc = Y(m1 + 2);
        bmax = __builtin_fmax(bmax, __builtin_fabs(yc));
        wy = wy + __builtin_fma(yc, tc, __builtin_fma(ya, ta, yb * tb));
      }
    }
  }
  if (bmax == 0.0) return 0;  // DGELSD: B == 0 -> zero solution, numpy reports no residual
  if (!(bmax >= 0x1p-970 && bmax <= 0x1p970)) return -1;
  const double sb = f.ntau1 * wy;  // DLARF applies the reflector: some y[k] != 0
  auto B = [&](int k) { return __builtin_fma(sb, v1(k), Y(k)); };
  if (m == 2) {
    if (!need_solution) return 0;
    if (f.R.rank < 0) return -1;
    dlalsd2_b(f.R, B(0), B(1), slope, icpt);
    return f.R.rank == 2 ? 0 : -3;
  }
  const double sc = f.sc, s2 = f.s2;
  auto v2 = [&](int k) { return k == 0 ? 1.0 : __builtin_fma(sc, v1(k + 1), 1.0) * s2; };
  // pass C: DLARF(v2, tau2) on b[1:]
  const int lastv2 = f.lastv2;
  double sb2 = 0.0;
  bool b2_upd = false;
  if (f.tau2nz) {
    bool any = false;
    const double w2 = gemv_t1(lastv2, [&](int k) {
      const double bk = B(k + 1);
      any = any || bk != 0.0;
      return bk;
    }, v2);
    if (any) {
      sb2 = f.ntau2 * w2;
      b2_upd = true;
    }
  }
  auto B2 = [&](int k) {
    const double bk = B(k);
    return (b2_upd && k - 1 < lastv2) ? __builtin_fma(sb2, v2(k - 1), bk) : bk;
  };
  double res = 0.0;
  if (need_ssr)
    for (int k = 2; k < m; k++) {
      const double bk = B2(k);
      res = res + bk * bk;
    }
  int rank = 2;
  if (need_solution) {
    if (f.R.rank < 0) return -1;
    dlalsd2_b(f.R, B(0), B2(1), slope, icpt);
    rank = f.R.rank;
  }
  ssr = rank == 2 ? res : 0.0;
  return rank == 2 ? 0 : -3;
}

// lsq_apply's solution for 2 <= m <= 4 as straight-line code: the same operations in the same
// order (pass A's four interleaved sums or its FMA tail, B = H1 y, pass C's gemv_t1 over
// lastv2 <= 3 elements, DLALSD's solve), with m selecting between them instead of loops and
// branches on per-lane counts, so a wave whose lanes fit segments of different short lengths
// runs one short sequence. The vertex fits (vertices2eqns, utils.py:646-669) are nearly all
// 2-4 points long. tests/test_lapack_emulation.py checks it against lsq_apply bit for bit.
template <class GX, class GY>
__host__ __device__ inline int lsq_apply_small(const lsq_xf& f, GX X, GY Y, double& slope,
                                               double& icpt) {
  slope = 0.0;
  icpt = 0.0;
  if (f.rc < 0) return f.rc;
  const int m = f.m;
  const double s1 = f.s1;
  const bool m3p = m >= 3, m4 = m >= 4;
  const double y0 = Y(0), y1 = Y(1), y2 = m3p ? Y(2) : 0.0, y3 = m4 ? Y(3) : 0.0;
  const double t1 = (double)X(1) * s1;
  const double t2 = m3p ? (double)X(2) * s1 : 0.0;
  const double t3 = m4 ? (double)X(3) * s1 : 0.0;
  // pass A, y half (lsq_apply: m1 = 4 for m = 4, else the FMA tail)
  double wy;
  if (m4) {
    const double Q0 = 0.0 + y0 * 1.0, Q1 = 0.0 + y1 * t1, Q2 = 0.0 + y2 * t2, Q3 = 0.0 + y3 * t3;
    wy = __builtin_fma((Q0 + Q2) + (Q1 + Q3), 1.0, 0.0);
  } else {
    const double inner = __builtin_fma(y0, 1.0, y1 * t1);
    wy = 0.0 + (m3p ? __builtin_fma(y2, t2, inner) : inner);
  }
  const double bmax = __builtin_fmax(__builtin_fmax(__builtin_fabs(y0), __builtin_fabs(y1)),
                                     __builtin_fmax(__builtin_fabs(y2), __builtin_fabs(y3)));
  if (bmax == 0.0) return 0;  // DGELSD: B == 0 -> zero solution
  if (!(bmax >= 0x1p-970 && bmax <= 0x1p970)) return -1;
  const double sb = f.ntau1 * wy;
  const double B0 = __builtin_fma(sb, 1.0, y0), B1 = __builtin_fma(sb, t1, y1);
  double b1 = B1;
  if (m3p) {
    const double B2 = __builtin_fma(sb, t2, y2), B3 = __builtin_fma(sb, t3, y3);
    if (f.tau2nz) {  // pass C: gemv_t1(lastv2, B(k+1), v2) and DLARF's "any nonzero" test
      const double sc = f.sc, s2 = f.s2;
      const int lv = f.lastv2;
      const double v21 = __builtin_fma(sc, t2, 1.0) * s2;
      const double v22 = m4 ? __builtin_fma(sc, t3, 1.0) * s2 : 0.0;
      double w2;
      bool any;
      if (lv == 1) {
        w2 = __builtin_fma(B1, 1.0, 0.0);
        any = B1 != 0.0;
      } else if (lv == 2) {
        w2 = 0.0 + __builtin_fma(B1, 1.0, B2 * v21);
        any = B1 != 0.0 || B2 != 0.0;
      } else {
        w2 = 0.0 + __builtin_fma(B3, v22, __builtin_fma(B1, 1.0, B2 * v21));
        any = B1 != 0.0 || B2 != 0.0 || B3 != 0.0;
      }
      if (any) b1 = __builtin_fma(f.ntau2 * w2, 1.0, B1);
    }
  }
  if (f.R.rank < 0) return -1;
  dlalsd2_b(f.R, B0, b1, slope, icpt);
  return f.R.rank == 2 ? 0 : -3;
}

template <class GX, class GY>
__host__ __device__ inline int lstsq_xint(int m, GX X, GY Y, bool need_solution, bool need_ssr,
                                          double& slope, double& icpt, double& ssr) {
  lsq_xf f;
  lsq_factor(m, X, f);
  return lsq_apply(f, X, Y, need_solution, need_ssr, slope, icpt, ssr);
}

// ------------------------------------------------------------------------------------------------
// Table of lsq_factor results for the x-sets segments usually have (year offsets < 64): m = 2
// with a gap <= 16, m = 3 with gaps <= 8, m = 4 with gaps <= 4, and m >= 5 consecutive years.
// Built on the device once per context (lt_abi.hip); lookups that miss factor on the fly. (Slots
// for 5-8 point x-sets with gaps of 1-2 years were tried: the key's loop, inlined into the
// year-major output loop, spilled 29 VGPRs of the c5 instance, 986 vs 1190 Mpx/s,
// profiles/r03_ab6; taken only in the miss branch it still spilled 14.)
// ------------------------------------------------------------------------------------------------
constexpr int kXtM2 = 0, kXtM3 = 64 * 16, kXtM4 = kXtM3 + 64 * 64, kXtCons = kXtM4 + 64 * 64,
              kXtSize = kXtCons + 64 * 64;

// table slot of the x-set X(0) < ... < X(m-1) (all < 64), or -1
template <class GX>
__host__ __device__ inline int xset_key(int m, GX X) {
  const int x0 = X(0);
  if (x0 < 0 || x0 > 63) return -1;
  if (m == 2) {
    const int d = X(1) - x0;
    return (d >= 1 && d <= 16) ? kXtM2 + x0 * 16 + (d - 1) : -1;
  }
  if (m == 3) {
    const int x1 = X(1), d1 = x1 - x0, d2 = X(2) - x1;
    return (d1 >= 1 && d1 <= 8 && d2 >= 1 && d2 <= 8) ? kXtM3 + x0 * 64 + (d1 - 1) * 8 + (d2 - 1)
                                                      : -1;
  }
  if (m == 4) {
    const int x1 = X(1), x2 = X(2), d1 = x1 - x0, d2 = x2 - x1, d3 = X(3) - x2;
    return (d1 >= 1 && d1 <= 4 && d2 >= 1 && d2 <= 4 && d3 >= 1 && d3 <= 4)
               ? kXtM4 + x0 * 64 + (d1 - 1) * 16 + (d2 - 1) * 4 + (d3 - 1)
               : -1;
  }
  if (m >= 5 && m <= 64 && X(m - 1) - x0 == m - 1) return kXtCons + x0 * 64 + (m - 1);
  return -1;
}

// the x-set of table slot idx: m and xs[0..m-1]; false for a slot no x-set maps to
__host__ __device__ inline bool xset_of_key(int idx, int& m, int* xs) {
  int d[3] = {1, 1, 1};
  if (idx < kXtM3) {
    m = 2;
    xs[0] = idx / 16;
    d[0] = idx % 16 + 1;
  } else if (idx < kXtM4) {
    const int r = idx - kXtM3;
    m = 3;
    xs[0] = r / 64;
    d[0] = (r / 8) % 8 + 1;
    d[1] = r % 8 + 1;
  } else if (idx < kXtCons) {
    const int r = idx - kXtM4;
    m = 4;
    xs[0] = r / 64;
    d[0] = (r / 16) % 4 + 1;
    d[1] = (r / 4) % 4 + 1;
    d[2] = r % 4 + 1;
  } else if (idx < kXtSize) {
    const int r = idx - kXtCons;
    m = r % 64 + 1;
    xs[0] = r / 64;
    if (m < 5) return false;
  } else {
    return false;
  }
  for (int k = 1; k < m; k++) xs[k] = xs[k - 1] + (m <= 4 ? d[k - 1] : 1);
  return xs[m - 1] <= 63;
}

}  // namespace lt
