// rcp_check.hip — the one hardware constant of the a-priori screening bounds (DESIGN.md §
// Screening bounds): the relative error of v_rcp_f64 (__builtin_amdgcn_rcp on binary64) and of
// the kernel's reciprocal, v_rcp_f64 plus one Newton step fma(r, fma(-d, r, 1), r) (lt_fast.h
// price, the labels-only fits). N random binary64 d over the ranges the kernels take reciprocals
// of (m*D <= 2^35, D, m: integers; plus random mantissas at every exponent in [0, 64]), checked
// on the host against 1/d in x87 extended precision. Prints one JSON object.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

__global__ void rcp_kernel(const double* d, double* r0, double* r1, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double x = d[i];
  const double a = __builtin_amdgcn_rcp(x);
  r0[i] = a;
  r1[i] = __builtin_fma(a, __builtin_fma(-x, a, 1.0), a);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : (1 << 24);
  std::mt19937_64 rng(12345);
  std::vector<double> d(n), r0(n), r1(n);
  for (int i = 0; i < n; i++) {
    if (i % 2 == 0) {  // integers as the kernels form them: m*D, D, m
      d[i] = (double)(1 + (rng() % (1ull << (1 + rng() % 35))));
    } else {  // random mantissa, exponent in [0, 64]
      const uint64_t mant = rng() & ((1ull << 52) - 1);
      const uint64_t ex = 1023 + rng() % 65;
      const uint64_t b = (ex << 52) | mant;
      memcpy(&d[i], &b, 8);
    }
  }
  double *dd, *d0, *d1;
  if (hipMalloc(&dd, n * 8) || hipMalloc(&d0, n * 8) || hipMalloc(&d1, n * 8)) return 1;
  if (hipMemcpy(dd, d.data(), n * 8, hipMemcpyHostToDevice)) return 1;
  hipLaunchKernelGGL(rcp_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, dd, d0, d1, n);
  if (hipMemcpy(r0.data(), d0, n * 8, hipMemcpyDeviceToHost)) return 1;
  if (hipMemcpy(r1.data(), d1, n * 8, hipMemcpyDeviceToHost)) return 1;
  long double e0 = 0, e1 = 0;
  double w0 = 0, w1 = 0;
  for (int i = 0; i < n; i++) {
    const long double ex = 1.0L / (long double)d[i];
    const long double a = fabsl(((long double)r0[i] - ex) / ex);
    const long double b = fabsl(((long double)r1[i] - ex) / ex);
    if (a > e0) { e0 = a; w0 = d[i]; }
    if (b > e1) { e1 = b; w1 = d[i]; }
  }
  printf("{\"n\": %d, \"rcp_max_rel_err\": %.6Le, \"rcp_log2\": %.3f, \"rcp_worst_d\": %.17g, "
         "\"rcp_newton_max_rel_err\": %.6Le, \"rcp_newton_log2\": %.3f, \"rcp_newton_worst_d\": "
         "%.17g, \"unit_roundoff_log2\": -53}\n",
         n, e0, (double)log2l(e0 > 0 ? e0 : 1e-300L), w0, e1,
         (double)log2l(e1 > 0 ? e1 : 1e-300L), w1);
  return 0;
}
