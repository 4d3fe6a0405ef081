// vgpr_edge.hip — do binary64 VALU results written to the last register pair of a wave's VGPR
// allocation come back intact? (debugging aid for the wrong-result variants, DESIGN.md
// § Wrong-result variants: the failing c3 code object is bit-exact with its allocation raised from
// 128 to 136 VGPRs, same code, and only it of the analyze instances writes v[126:127] with
// binary64 ops: v_mul_f64, v_add_f64, v_max_f64, v_cvt_f64_{i32,u32}.)
//
// Every lane iterates x <- fl(fl(x * m) + a), N times, in one asm block whose accumulator is the
// pair named by PAIR (v[126:127]: the allocation's last pair when nothing above v127 is used; or
// v[120:121] with v127 merely clobbered: the same 128-VGPR allocation, the pair not at its end).
// Each lane's inputs depend on its lane only, so every wave must produce the same 64 values; the
// host compares each wave with a host reference of the same roundings and counts mismatching
// lanes. A code object's allocation can be raised in place (tools/co_patch.py --vgprs) for the
// same code at another allocation.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build/bin/vgpr_edge tools/vgpr_edge.hip
//   vgpr_edge WAVES ITERS  -> one JSON line per kernel
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define EDGE_BODY(PAIR, ...)                                                                    \
  const int lane = threadIdx.x;                                                                \
  double x = 1.0 + lane * 0x1p-6, m = 1.0 + 0x1p-20 * (lane + 1), a = -0x1p-9 * (lane + 3);     \
  uint32_t cnt = iters;                                                                        \
  double r;                                                                                    \
  asm volatile("v_mov_b64 " PAIR ", %[x]\n"                                                    \
               "1:\n"                                                                          \
               "v_mul_f64 " PAIR ", " PAIR ", %[m]\n"                                          \
               "v_add_f64 " PAIR ", " PAIR ", %[a]\n"                                          \
               "s_sub_u32 %[c], %[c], 1\n"                                                     \
               "s_cmp_lg_u32 %[c], 0\n"                                                        \
               "s_cbranch_scc1 1b\n"                                                           \
               "v_mov_b64 %[r], " PAIR "\n"                                                    \
               : [r] "=&v"(r), [c] "+s"(cnt)                                                   \
               : [x] "v"(x), [m] "v"(m), [a] "v"(a)                                            \
               : __VA_ARGS__, "scc");                                                               \
  out[(size_t)blockIdx.x * 64 + lane] = r;

// the pair at the allocation's end: the asm names v126, v127 and nothing higher
__global__ __launch_bounds__(64, 4) void edge_kernel(double* out, uint32_t iters) {
  EDGE_BODY("v[126:127]", "v126", "v127")
}
// control: the same allocation (v127 clobbered), the accumulator pair inside it
__global__ __launch_bounds__(64, 4) void inner_kernel(double* out, uint32_t iters) {
  EDGE_BODY("v[120:121]", "v120", "v121", "v127")
}

static double reference(int lane, uint32_t iters) {
  volatile double x = 1.0 + lane * 0x1p-6, m = 1.0 + 0x1p-20 * (lane + 1),
                  a = -0x1p-9 * (lane + 3);
  for (uint32_t i = 0; i < iters; i++) {
    volatile double p = x * m;
    x = p + a;
  }
  return x;
}

template <class K>
static int run(const char* name, K kern, int waves, uint32_t iters) {
  double* d = nullptr;
  if (hipMalloc(&d, sizeof(double) * 64 * (size_t)waves) != hipSuccess) return 1;
  hipLaunchKernelGGL(kern, dim3(waves), dim3(64), 0, 0, d, iters);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<double> h((size_t)64 * waves);
  if (hipMemcpy(h.data(), d, sizeof(double) * h.size(), hipMemcpyDeviceToHost) != hipSuccess)
    return 3;
  double ref[64];
  for (int l = 0; l < 64; l++) ref[l] = reference(l, iters);
  long bad_lanes = 0, bad_waves = 0, first = -1;
  for (int w = 0; w < waves; w++) {
    int b = 0;
    for (int l = 0; l < 64; l++)
      if (memcmp(&h[(size_t)w * 64 + l], &ref[l], 8) != 0) b++;
    bad_lanes += b;
    if (b) {
      bad_waves++;
      if (first < 0) first = w;
    }
  }
  printf("{\"kernel\": \"%s\", \"waves\": %d, \"iters\": %u, \"mismatching_lanes\": %ld, "
         "\"mismatching_waves\": %ld, \"first_bad_wave\": %ld}\n",
         name, waves, iters, bad_lanes, bad_waves, first);
  (void)hipFree(d);
  return 0;
}

int main(int argc, char** argv) {
  const int waves = argc > 1 ? atoi(argv[1]) : 262144;
  const uint32_t iters = argc > 2 ? (uint32_t)atoi(argv[2]) : 1000;
  if (waves <= 0 || waves > (1 << 22) || iters == 0) return 4;
  int rc = run("edge_v126_127", edge_kernel, waves, iters);
  if (rc == 0) rc = run("inner_v120_121", inner_kernel, waves, iters);
  return rc;
}
