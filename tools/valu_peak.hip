// valu_peak.hip — measured VALU issue peak of one MI355X SIMD.
//
// The analyze kernel is bound by vector-instruction issue, so its roofline needs the rate at which
// one SIMD issues wave64 VALU instructions of the kernel's own classes, at its own occupancy. This
// program measures it with no memory traffic in the timed loop: each wave runs ITERS iterations of
// a straight-line stream of register-only instructions (inline asm, eight independent chains per
// class so no instruction waits on its predecessor), and the launch time gives wave-instructions
// per second per SIMD; an s_memtime bracket per wave gives shader cycles per instruction.
//
// Occupancy is pinned with dynamic LDS: one wave per workgroup, 160 KiB / (4 W) bytes each, so at
// most W waves share a SIMD (4 W per CU). Kinds:
//   add_u32, cndmask, cmp (32-bit VALU), fma_f32, add_f64, fma_f64, mul_f64, rcp_f64,
//   lshl_b64 (64-bit integer), mix_c2 (the analyze kernel's c2 PMC mix, profiles/r0?_pmc_c2.json:
//   21 % FP64, 1.5 % INT64, the rest 32-bit, plus half as many SALU instructions as VALU).
// Output: one JSON object on stdout. Nothing here stores through the scalar cache: results leave
// through ordinary vector global stores.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

// Round-5 kinds (the forms the compiler emits most in the c2 kernel):
//   cndmask_b32_vcc       e32 selects on VCC, VCC written by an s_mov_b64 each iteration (round 4:
//                         22.9 cycles at every occupancy, unexplained)
//   cndmask_vcc_valu      e32 selects on VCC, VCC written ONCE per iteration by a VOPC e32 compare
//   cmp_cndmask_vcc       the compiler's pair: v_cmp_*_e32 (VCC) then v_cndmask_b32_e32, eight
//                         independent pairs per block (one VCC: each pair waits on its compare)
//   cndmask_e64_vcc       e64 selects naming vcc as the mask, VCC written by s_mov each iteration
//   cndmask_e64_smov      e64 selects on an SGPR pair written by s_mov each iteration (is it the
//                         SALU write of a mask, or VCC itself?)
//   cndmask_e64_vcmp      e64 selects on an SGPR pair written by a VOPC e64 compare each iteration
//   mov_b64               v_mov_b64 (gfx950's 64-bit move)
//   cmp_e32               VOPC e32 compares writing VCC (back to back)
//   nop_mix               one s_nop 0 per eight v_add_u32 (the hazard padding the compiler emits)
// Round-5 second set (e32 selects on a VCC not written by the instruction before them measured 16
// cycles, VALU-written, and 23, SALU-written; the compiler's compare -> select pair 4.1):
//   cmp_cnd2_vcc          v_cmp_e32 (VCC) then TWO e32 selects on it (a binary64 select), 8 chains
//   cmp_cnd4_vcc          v_cmp_e32 (VCC) then FOUR e32 selects on it
//   cmp_gap_cnd_vcc       v_cmp_e32 (VCC), three independent v_add_u32, then one e32 select
//   cmp64_cnd2            v_cmp_e64 into an SGPR pair, then two e64 selects on it
enum Kind { ADD_U32, CNDMASK, CMP, FMA_F32, FMA_F32K, ADD_F64, FMA_F64, MUL_F64, RCP_F64, LSHL_B64,
            MIX_C2, MOV_B32, CNDMASK_VCC, CNDMASK_VCC_VALU, CMP_CNDMASK_VCC, CNDMASK_E64_VCC,
            CNDMASK_E64_SMOV, CNDMASK_E64_VCMP, MOV_B64, CMP_E32, NOP_MIX, CMP_CND2_VCC,
            CMP_CND4_VCC, CMP_GAP_CND_VCC, CMP64_CND2, MAD_U64, MAD_U24, MUL_LO, NKIND };
static const char* kKindName[NKIND] = {"add_u32", "cndmask_b32", "cmp_gt_u32", "fma_f32",
                                       "fma_f32_k", "add_f64", "fma_f64", "mul_f64", "rcp_f64",
                                       "lshlrev_b64", "mix_c2", "mov_b32", "cndmask_b32_vcc",
                                       "cndmask_vcc_valu", "cmp_cndmask_vcc", "cndmask_e64_vcc",
                                       "cndmask_e64_smov", "cndmask_e64_vcmp", "mov_b64",
                                       "cmp_e32", "nop_mix", "cmp_cnd2_vcc", "cmp_cnd4_vcc",
                                       "cmp_gap_cnd_vcc", "cmp64_cnd2", "mad_u64_u32", "mad_u32_u24",
                                       "mul_lo_u32"};
// VALU / SALU instructions per loop iteration of each kind (the asm blocks below)
static const int kValuPerIter[NKIND] = {64, 64, 64, 64, 64, 64, 64, 64, 32, 64, 103, 64, 64,
                                        65, 64, 64, 64, 65, 64, 64, 64, 48, 80, 80, 48, 64, 64, 64};
static const int kSaluPerIter[NKIND] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 50, 0, 1,
                                        0, 0, 1, 1, 0, 0, 0, 8, 0, 0, 0, 0, 0, 0, 0};

#define R8(s) s s s s s s s s

template <int K>
__global__ void __launch_bounds__(64) valu_kernel(unsigned* out, unsigned long long* cyc, int iters) {
  extern __shared__ unsigned lds_pad[];  // occupancy only
  const unsigned t = threadIdx.x + blockIdx.x * 64u;
  unsigned a0 = t, a1 = t + 1, a2 = t + 2, a3 = t + 3, a4 = t + 4, a5 = t + 5, a6 = t + 6, a7 = t + 7;
  const unsigned inc = (t & 3) + 1;
  float f0 = a0, f1 = a1, f2 = a2, f3 = a3, f4 = a4, f5 = a5, f6 = a6, f7 = a7;
  const float fm = 1.0000001f, fa = 0.5f;
  double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7;
  const double dm = 1.0000000001, da = 0.25;
  unsigned long long q0 = a0, q1 = a1, q2 = a2, q3 = a3, q4 = a4, q5 = a5, q6 = a6, q7 = a7;
  unsigned long long m0 = 0, m1 = 0, m2 = 0, m3 = 0, m4 = 0, m5 = 0, m6 = 0, m7 = 0;
  const unsigned long long sel = (blockIdx.x & 1) ? ~0ull : 0x5555555555555555ull;
  unsigned s0 = 1, s1 = 2, s2 = 3, s3 = 4;
  if (lds_pad[0] == 0xdeadbeefu && t == 0xffffffffu) a0 = 0;  // keeps the LDS allocation
  unsigned long long c0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c0)::"memory");
  for (int it = 0; it < iters; it++) {
    if constexpr (K == ADD_U32) {
      asm volatile(R8("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                      "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(inc));
    } else if constexpr (K == CNDMASK) {
      asm volatile(R8("v_cndmask_b32_e64 %0, %0, %8, %9\n v_cndmask_b32_e64 %1, %1, %8, %9\n"
                      "v_cndmask_b32_e64 %2, %2, %8, %9\n v_cndmask_b32_e64 %3, %3, %8, %9\n"
                      "v_cndmask_b32_e64 %4, %4, %8, %9\n v_cndmask_b32_e64 %5, %5, %8, %9\n"
                      "v_cndmask_b32_e64 %6, %6, %8, %9\n v_cndmask_b32_e64 %7, %7, %8, %9\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(inc), "s"(sel));
    } else if constexpr (K == CMP) {
      asm volatile(R8("v_cmp_gt_u32_e64 %0, %8, %9\n v_cmp_gt_u32_e64 %1, %8, %10\n"
                      "v_cmp_gt_u32_e64 %2, %8, %11\n v_cmp_gt_u32_e64 %3, %8, %12\n"
                      "v_cmp_gt_u32_e64 %4, %8, %13\n v_cmp_gt_u32_e64 %5, %8, %14\n"
                      "v_cmp_gt_u32_e64 %6, %8, %15\n v_cmp_gt_u32_e64 %7, %8, %9\n")
                   : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3), "=s"(m4), "=s"(m5), "=s"(m6), "=s"(m7)
                   : "v"(inc), "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6));
      a7 += (unsigned)(m0 ^ m1 ^ m2 ^ m3 ^ m4 ^ m5 ^ m6 ^ m7);
    } else if constexpr (K == FMA_F32) {
      asm volatile(R8("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n"
                      "v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n"
                      "v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9\n")
                   : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7)
                   : "v"(fm), "v"(fa));
    } else if constexpr (K == MOV_B32) {  // VOP1 moves (a rotation of eight registers)
      asm volatile(R8("v_mov_b32 %0, %1\n v_mov_b32 %1, %2\n v_mov_b32 %2, %3\n v_mov_b32 %3, %4\n"
                      "v_mov_b32 %4, %5\n v_mov_b32 %5, %6\n v_mov_b32 %6, %7\n v_mov_b32 %7, %0\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if constexpr (K == CNDMASK_VCC) {  // VOP2 selects on VCC (the e32 form)
      asm volatile("s_mov_b64 vcc, %9\n"
                   R8("v_cndmask_b32_e32 %0, %0, %8, vcc\n v_cndmask_b32_e32 %1, %1, %8, vcc\n"
                      "v_cndmask_b32_e32 %2, %2, %8, vcc\n v_cndmask_b32_e32 %3, %3, %8, vcc\n"
                      "v_cndmask_b32_e32 %4, %4, %8, vcc\n v_cndmask_b32_e32 %5, %5, %8, vcc\n"
                      "v_cndmask_b32_e32 %6, %6, %8, vcc\n v_cndmask_b32_e32 %7, %7, %8, vcc\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(inc), "s"(sel)
                   : "vcc");
    } else if constexpr (K == CNDMASK_VCC_VALU) {  // VCC from one VOPC e32 compare per iteration
      asm volatile("v_cmp_gt_u32_e32 vcc, %8, %9\n"
                   R8("v_cndmask_b32_e32 %0, %0, %8, vcc\n v_cndmask_b32_e32 %1, %1, %8, vcc\n"
                      "v_cndmask_b32_e32 %2, %2, %8, vcc\n v_cndmask_b32_e32 %3, %3, %8, vcc\n"
                      "v_cndmask_b32_e32 %4, %4, %8, vcc\n v_cndmask_b32_e32 %5, %5, %8, vcc\n"
                      "v_cndmask_b32_e32 %6, %6, %8, vcc\n v_cndmask_b32_e32 %7, %7, %8, vcc\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(inc), "v"(t)
                   : "vcc");
    } else if constexpr (K == CMP_CNDMASK_VCC) {  // compare (VCC) -> select pairs, eight chains
#define CC8 "v_cmp_gt_u32_e32 vcc, %8, %0\n v_cndmask_b32_e32 %0, %0, %8, vcc\n" \
            "v_cmp_gt_u32_e32 vcc, %8, %1\n v_cndmask_b32_e32 %1, %1, %8, vcc\n" \
            "v_cmp_gt_u32_e32 vcc, %8, %2\n v_cndmask_b32_e32 %2, %2, %8, vcc\n" \
            "v_cmp_gt_u32_e32 vcc, %8, %3\n v_cndmask_b32_e32 %3, %3, %8, vcc\n" \
            "v_cmp_gt_u32_e32 vcc, %8, %4\n v_cndmask_b32_e32 %4, %4, %8, vcc\n" \
            "v_cmp_gt_u32_e32 vcc, %8, %5\n v_cndmask_b32_e32 %5, %5, %8, vcc\n" \
            "v_cmp_gt_u32_e32 vcc, %8, %6\n v_cndmask_b32_e32 %6, %6, %8, vcc\n" \
            "v_cmp_gt_u32_e32 vcc, %8, %7\n v_cndmask_b32_e32 %7, %7, %8, vcc\n"
      asm volatile(CC8 CC8 CC8 CC8
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(inc)
                   : "vcc");
#undef CC8
    } else if constexpr (K == CNDMASK_E64_VCC) {  // e64 selects naming vcc, VCC from s_mov
      asm volatile("s_mov_b64 vcc, %9\n"
                   R8("v_cndmask_b32_e64 %0, %0, %8, vcc\n v_cndmask_b32_e64 %1, %1, %8, vcc\n"
                      "v_cndmask_b32_e64 %2, %2, %8, vcc\n v_cndmask_b32_e64 %3, %3, %8, vcc\n"
                      "v_cndmask_b32_e64 %4, %4, %8, vcc\n v_cndmask_b32_e64 %5, %5, %8, vcc\n"
                      "v_cndmask_b32_e64 %6, %6, %8, vcc\n v_cndmask_b32_e64 %7, %7, %8, vcc\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(inc), "s"(sel)
                   : "vcc");
    } else if constexpr (K == CNDMASK_E64_SMOV) {  // e64 selects on an SGPR pair from s_mov
      asm volatile("s_mov_b64 %8, %10\n"
                   R8("v_cndmask_b32_e64 %0, %0, %9, %8\n v_cndmask_b32_e64 %1, %1, %9, %8\n"
                      "v_cndmask_b32_e64 %2, %2, %9, %8\n v_cndmask_b32_e64 %3, %3, %9, %8\n"
                      "v_cndmask_b32_e64 %4, %4, %9, %8\n v_cndmask_b32_e64 %5, %5, %9, %8\n"
                      "v_cndmask_b32_e64 %6, %6, %9, %8\n v_cndmask_b32_e64 %7, %7, %9, %8\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7),
                     "+s"(m0)
                   : "v"(inc), "s"(sel));
    } else if constexpr (K == CNDMASK_E64_VCMP) {  // e64 selects on an SGPR pair from a VOPC e64
      asm volatile("v_cmp_gt_u32_e64 %8, %9, %10\n"
                   R8("v_cndmask_b32_e64 %0, %0, %9, %8\n v_cndmask_b32_e64 %1, %1, %9, %8\n"
                      "v_cndmask_b32_e64 %2, %2, %9, %8\n v_cndmask_b32_e64 %3, %3, %9, %8\n"
                      "v_cndmask_b32_e64 %4, %4, %9, %8\n v_cndmask_b32_e64 %5, %5, %9, %8\n"
                      "v_cndmask_b32_e64 %6, %6, %9, %8\n v_cndmask_b32_e64 %7, %7, %9, %8\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7),
                     "+s"(m0)
                   : "v"(inc), "v"(t));
    } else if constexpr (K == MAD_U64) {  // the 32 x 32 + 64 multiply-add the compiler uses for
      // an int32 a*a + s whose operands it cannot prove 24-bit (the DP's Sxx += x*x)
      asm volatile(R8("v_mad_u64_u32 %0, %8, %9, %9, %0\n v_mad_u64_u32 %1, %8, %9, %9, %1\n"
                      "v_mad_u64_u32 %2, %8, %9, %9, %2\n v_mad_u64_u32 %3, %8, %9, %9, %3\n"
                      "v_mad_u64_u32 %4, %8, %9, %9, %4\n v_mad_u64_u32 %5, %8, %9, %9, %5\n"
                      "v_mad_u64_u32 %6, %8, %9, %9, %6\n v_mad_u64_u32 %7, %8, %9, %9, %7\n")
                   : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(q4), "+v"(q5), "+v"(q6), "+v"(q7),
                     "=s"(m1)
                   : "v"(inc));
    } else if constexpr (K == MAD_U24) {  // the full-rate 24-bit multiply-add
      asm volatile(R8("v_mad_u32_u24 %0, %8, %8, %0\n v_mad_u32_u24 %1, %8, %8, %1\n"
                      "v_mad_u32_u24 %2, %8, %8, %2\n v_mad_u32_u24 %3, %8, %8, %3\n"
                      "v_mad_u32_u24 %4, %8, %8, %4\n v_mad_u32_u24 %5, %8, %8, %5\n"
                      "v_mad_u32_u24 %6, %8, %8, %6\n v_mad_u32_u24 %7, %8, %8, %7\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(inc));
    } else if constexpr (K == MUL_LO) {  // v_mul_lo_u32 (32 x 32, low half)
      asm volatile(R8("v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n"
                      "v_mul_lo_u32 %3, %3, %8\n v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n"
                      "v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(inc));
    } else if constexpr (K == MOV_B64) {  // 64-bit moves (a rotation of eight register pairs)
      asm volatile(R8("v_mov_b64 %0, %1\n v_mov_b64 %1, %2\n v_mov_b64 %2, %3\n v_mov_b64 %3, %4\n"
                      "v_mov_b64 %4, %5\n v_mov_b64 %5, %6\n v_mov_b64 %6, %7\n v_mov_b64 %7, %0\n")
                   : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(q4), "+v"(q5), "+v"(q6), "+v"(q7));
    } else if constexpr (K == CMP_E32) {  // VOPC e32 compares writing VCC, back to back
      asm volatile(R8("v_cmp_gt_u32_e32 vcc, %8, %0\n v_cmp_gt_u32_e32 vcc, %8, %1\n"
                      "v_cmp_gt_u32_e32 vcc, %8, %2\n v_cmp_gt_u32_e32 vcc, %8, %3\n"
                      "v_cmp_gt_u32_e32 vcc, %8, %4\n v_cmp_gt_u32_e32 vcc, %8, %5\n"
                      "v_cmp_gt_u32_e32 vcc, %8, %6\n v_cmp_gt_u32_e32 vcc, %8, %7\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(inc)
                   : "vcc");
    } else if constexpr (K == NOP_MIX) {  // an s_nop 0 after every eight 32-bit adds
      asm volatile(R8("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                      "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
                      "s_nop 0\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(inc));
    } else if constexpr (K == CMP_CND2_VCC) {  // compare, then a pair of selects on its VCC
#define P2(a, b) "v_cmp_gt_u32_e32 vcc, %8, " a "\n v_cndmask_b32_e32 " a ", " a ", %8, vcc\n" \
                 " v_cndmask_b32_e32 " b ", " b ", %8, vcc\n"
      asm volatile(P2("%0", "%1") P2("%2", "%3") P2("%4", "%5") P2("%6", "%7")
                   P2("%1", "%0") P2("%3", "%2") P2("%5", "%4") P2("%7", "%6")
                   P2("%0", "%1") P2("%2", "%3") P2("%4", "%5") P2("%6", "%7")
                   P2("%1", "%0") P2("%3", "%2") P2("%5", "%4") P2("%7", "%6")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(inc)
                   : "vcc");
#undef P2
    } else if constexpr (K == CMP_CND4_VCC) {  // compare, then four selects on its VCC
#define P4(a, b, c, d) "v_cmp_gt_u32_e32 vcc, %8, " a "\n v_cndmask_b32_e32 " a ", " a ", %8, vcc\n" \
                       " v_cndmask_b32_e32 " b ", " b ", %8, vcc\n v_cndmask_b32_e32 " c ", " c \
                       ", %8, vcc\n v_cndmask_b32_e32 " d ", " d ", %8, vcc\n"
      asm volatile(P4("%0", "%1", "%2", "%3") P4("%4", "%5", "%6", "%7")
                   P4("%1", "%2", "%3", "%0") P4("%5", "%6", "%7", "%4")
                   P4("%2", "%3", "%0", "%1") P4("%6", "%7", "%4", "%5")
                   P4("%3", "%0", "%1", "%2") P4("%7", "%4", "%5", "%6")
                   P4("%0", "%1", "%2", "%3") P4("%4", "%5", "%6", "%7")
                   P4("%1", "%2", "%3", "%0") P4("%5", "%6", "%7", "%4")
                   P4("%2", "%3", "%0", "%1") P4("%6", "%7", "%4", "%5")
                   P4("%3", "%0", "%1", "%2") P4("%7", "%4", "%5", "%6")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(inc)
                   : "vcc");
#undef P4
    } else if constexpr (K == CMP_GAP_CND_VCC) {  // compare, three independent adds, one select
#define G1(a, x, y, z) "v_cmp_gt_u32_e32 vcc, %8, " a "\n v_add_u32 " x ", " x ", %8\n" \
                       " v_add_u32 " y ", " y ", %8\n v_add_u32 " z ", " z ", %8\n" \
                       " v_cndmask_b32_e32 " a ", " a ", %8, vcc\n"
      asm volatile(G1("%0", "%1", "%2", "%3") G1("%4", "%5", "%6", "%7")
                   G1("%1", "%2", "%3", "%0") G1("%5", "%6", "%7", "%4")
                   G1("%2", "%3", "%0", "%1") G1("%6", "%7", "%4", "%5")
                   G1("%3", "%0", "%1", "%2") G1("%7", "%4", "%5", "%6")
                   G1("%0", "%1", "%2", "%3") G1("%4", "%5", "%6", "%7")
                   G1("%1", "%2", "%3", "%0") G1("%5", "%6", "%7", "%4")
                   G1("%2", "%3", "%0", "%1") G1("%6", "%7", "%4", "%5")
                   G1("%3", "%0", "%1", "%2") G1("%7", "%4", "%5", "%6")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(inc)
                   : "vcc");
#undef G1
    } else if constexpr (K == CMP64_CND2) {  // e64 compare into an SGPR pair, two e64 selects
#define Q2(a, b) "v_cmp_gt_u32_e64 %8, %9, " a "\n v_cndmask_b32_e64 " a ", " a ", %9, %8\n" \
                 " v_cndmask_b32_e64 " b ", " b ", %9, %8\n"
      asm volatile(Q2("%0", "%1") Q2("%2", "%3") Q2("%4", "%5") Q2("%6", "%7")
                   Q2("%1", "%0") Q2("%3", "%2") Q2("%5", "%4") Q2("%7", "%6")
                   Q2("%0", "%1") Q2("%2", "%3") Q2("%4", "%5") Q2("%6", "%7")
                   Q2("%1", "%0") Q2("%3", "%2") Q2("%5", "%4") Q2("%7", "%6")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7),
                     "=&s"(m0)
                   : "v"(inc));
#undef Q2
    } else if constexpr (K == FMA_F32K) {  // two VGPR sources and an inline constant
      asm volatile(R8("v_fma_f32 %0, %0, %8, 0.5\n v_fma_f32 %1, %1, %8, 0.5\n v_fma_f32 %2, %2, %8, 0.5\n"
                      "v_fma_f32 %3, %3, %8, 0.5\n v_fma_f32 %4, %4, %8, 0.5\n v_fma_f32 %5, %5, %8, 0.5\n"
                      "v_fma_f32 %6, %6, %8, 0.5\n v_fma_f32 %7, %7, %8, 0.5\n")
                   : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7)
                   : "v"(fm));
    } else if constexpr (K == ADD_F64) {
      asm volatile(R8("v_add_f64 %0, %0, %8\n v_add_f64 %1, %1, %8\n v_add_f64 %2, %2, %8\n"
                      "v_add_f64 %3, %3, %8\n v_add_f64 %4, %4, %8\n v_add_f64 %5, %5, %8\n"
                      "v_add_f64 %6, %6, %8\n v_add_f64 %7, %7, %8\n")
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                   : "v"(da));
    } else if constexpr (K == FMA_F64) {
      asm volatile(R8("v_fma_f64 %0, %0, %8, %9\n v_fma_f64 %1, %1, %8, %9\n v_fma_f64 %2, %2, %8, %9\n"
                      "v_fma_f64 %3, %3, %8, %9\n v_fma_f64 %4, %4, %8, %9\n v_fma_f64 %5, %5, %8, %9\n"
                      "v_fma_f64 %6, %6, %8, %9\n v_fma_f64 %7, %7, %8, %9\n")
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                   : "v"(dm), "v"(da));
    } else if constexpr (K == MUL_F64) {
      asm volatile(R8("v_mul_f64 %0, %0, %8\n v_mul_f64 %1, %1, %8\n v_mul_f64 %2, %2, %8\n"
                      "v_mul_f64 %3, %3, %8\n v_mul_f64 %4, %4, %8\n v_mul_f64 %5, %5, %8\n"
                      "v_mul_f64 %6, %6, %8\n v_mul_f64 %7, %7, %8\n")
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                   : "v"(dm));
    } else if constexpr (K == RCP_F64) {
      asm volatile("v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3\n"
                   "v_rcp_f64 %4, %4\n v_rcp_f64 %5, %5\n v_rcp_f64 %6, %6\n v_rcp_f64 %7, %7\n"
                   "v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3\n"
                   "v_rcp_f64 %4, %4\n v_rcp_f64 %5, %5\n v_rcp_f64 %6, %6\n v_rcp_f64 %7, %7\n"
                   "v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3\n"
                   "v_rcp_f64 %4, %4\n v_rcp_f64 %5, %5\n v_rcp_f64 %6, %6\n v_rcp_f64 %7, %7\n"
                   "v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3\n"
                   "v_rcp_f64 %4, %4\n v_rcp_f64 %5, %5\n v_rcp_f64 %6, %6\n v_rcp_f64 %7, %7\n"
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7));
    } else if constexpr (K == LSHL_B64) {
      asm volatile(R8("v_lshlrev_b64 %0, 1, %0\n v_lshlrev_b64 %1, 1, %1\n v_lshlrev_b64 %2, 1, %2\n"
                      "v_lshlrev_b64 %3, 1, %3\n v_lshlrev_b64 %4, 1, %4\n v_lshlrev_b64 %5, 1, %5\n"
                      "v_lshlrev_b64 %6, 1, %6\n v_lshlrev_b64 %7, 1, %7\n")
                   : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(q4), "+v"(q5), "+v"(q6), "+v"(q7));
    } else {  // MIX_C2: five blocks of the c2 analyze kernel's PMC mix
#define MIXBLK(ADDF, LSH)                                                              \
  asm volatile(ADDF                                                                    \
               "v_fma_f64 %1, %1, %13, %14\n v_add_u32 %4, %4, %15\n"                  \
               "v_cndmask_b32_e64 %5, %5, %15, %16\n v_cmp_gt_u32_e64 %8, %15, %4\n"   \
               "v_add_u32 %6, %6, %15\n v_cndmask_b32_e64 %7, %7, %15, %16\n"          \
               "s_add_u32 %9, %9, 1\n s_and_b32 %10, %10, %9\n"                        \
               "v_bfe_u32 %5, %4, 3, 7\n v_mul_f64 %2, %2, %13\n"                      \
               "v_cndmask_b32_e64 %4, %4, %15, %16\n v_add_u32 %7, %7, %15\n"          \
               "s_add_u32 %11, %11, %9\n s_and_b32 %9, %9, %11\n"                      \
               "v_cndmask_b32_e64 %6, %6, %15, %16\n v_cmp_gt_u32_e64 %8, %15, %5\n"   \
               "v_add_f64 %3, %3, %14\n v_bfe_u32 %6, %7, 2, 9\n"                      \
               "s_add_u32 %10, %10, %11\n s_and_b32 %11, %11, %10\n"                   \
               "v_cndmask_b32_e64 %5, %5, %15, %16\n v_cndmask_b32_e64 %7, %7, %15, %16\n" \
               "v_cmp_gt_u32_e64 %8, %15, %6\n v_fma_f64 %1, %1, %13, %14\n"           \
               "s_add_u32 %9, %9, %10\n s_and_b32 %10, %10, %9\n"                      \
               "v_bfe_u32 %4, %5, 1, 11\n v_cndmask_b32_e64 %6, %6, %15, %16\n"        \
               LSH                                                                     \
               "s_add_u32 %11, %11, 3\n s_and_b32 %9, %9, %11\n"                       \
               : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(a0), "+v"(a1), "+v"(a2), \
                 "+v"(a3), "=s"(m0), "+s"(s0), "+s"(s1), "+s"(s2), "+v"(q0)            \
               : "v"(dm), "v"(da), "v"(inc), "s"(sel)                                 \
               : "scc")
      // per block: fma_f64 x2, mul_f64 x1, add_f64 x1, add_u32 x3, cndmask x8, cmp x3, bfe x3
      // = 20 VALU (+ one add_f64 in the first block, one lshlrev_b64 in two blocks), 10 SALU:
      // 103 VALU, 21 FP64 (20.4 %), 2 INT64 (1.9 %), 50 SALU per iteration
      MIXBLK("v_add_f64 %0, %0, %14\n", "");
      MIXBLK("", "v_lshlrev_b64 %12, 1, %12\n");
      MIXBLK("", "");
      MIXBLK("", "v_lshlrev_b64 %12, 1, %12\n");
      MIXBLK("", "");
#undef MIXBLK
    }
  }
  unsigned long long c1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c1)::"memory");
  unsigned r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ s0 ^ s1 ^ s2 ^ s3 ^ (unsigned)(m0 ^ q0 ^ q1 ^ q2 ^ q3 ^ q4 ^ q5 ^ q6 ^ q7);
  r ^= (unsigned)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7);
  r ^= (unsigned)(long long)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
  out[t] = r;  // vector store
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;  // vector store from lane 0
}

typedef void (*KFn)(unsigned*, unsigned long long*, int);
static KFn kernel_of(int k) {
  switch (k) {
    case ADD_U32: return valu_kernel<ADD_U32>;
    case CNDMASK: return valu_kernel<CNDMASK>;
    case CMP: return valu_kernel<CMP>;
    case FMA_F32: return valu_kernel<FMA_F32>;
    case FMA_F32K: return valu_kernel<FMA_F32K>;
    case MOV_B32: return valu_kernel<MOV_B32>;
    case CNDMASK_VCC: return valu_kernel<CNDMASK_VCC>;
    case ADD_F64: return valu_kernel<ADD_F64>;
    case FMA_F64: return valu_kernel<FMA_F64>;
    case MUL_F64: return valu_kernel<MUL_F64>;
    case RCP_F64: return valu_kernel<RCP_F64>;
    case LSHL_B64: return valu_kernel<LSHL_B64>;
    case MIX_C2: return valu_kernel<MIX_C2>;
    case CNDMASK_VCC_VALU: return valu_kernel<CNDMASK_VCC_VALU>;
    case CMP_CNDMASK_VCC: return valu_kernel<CMP_CNDMASK_VCC>;
    case CNDMASK_E64_VCC: return valu_kernel<CNDMASK_E64_VCC>;
    case CNDMASK_E64_SMOV: return valu_kernel<CNDMASK_E64_SMOV>;
    case CNDMASK_E64_VCMP: return valu_kernel<CNDMASK_E64_VCMP>;
    case MOV_B64: return valu_kernel<MOV_B64>;
    case CMP_E32: return valu_kernel<CMP_E32>;
    case NOP_MIX: return valu_kernel<NOP_MIX>;
    case CMP_CND2_VCC: return valu_kernel<CMP_CND2_VCC>;
    case CMP_CND4_VCC: return valu_kernel<CMP_CND4_VCC>;
    case CMP_GAP_CND_VCC: return valu_kernel<CMP_GAP_CND_VCC>;
    case CMP64_CND2: return valu_kernel<CMP64_CND2>;
    case MAD_U64: return valu_kernel<MAD_U64>;
    case MAD_U24: return valu_kernel<MAD_U24>;
    case MUL_LO: return valu_kernel<MUL_LO>;
    default: return valu_kernel<MIX_C2>;
  }
}

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 20000;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int simds = cus * 4;
  const size_t lds_cu = 160 * 1024;
  // one generation: every wave of the launch is resident from start to end, so the s_memtime
  // bracket of each wave spans W co-resident waves per SIMD throughout
  const int gens = 1;
  const int wps[] = {1, 2, 4, 8};
  const int max_waves = cus * 4 * 8 * gens;
  unsigned* out;
  unsigned long long* cyc;
  CHECK(hipMalloc(&out, (size_t)max_waves * 64 * sizeof(unsigned)));
  CHECK(hipMalloc(&cyc, (size_t)max_waves * sizeof(unsigned long long)));
  std::vector<unsigned long long> hc(max_waves);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("{\"device\": \"%s\", \"gcn_arch\": \"%s\", \"cus\": %d, \"simds\": %d, \"clock_khz\": %d, "
         "\"iters\": %d, \"generations\": %d, \"results\": [",
         prop.name, prop.gcnArchName, cus, simds, prop.clockRate, iters, gens);
  bool first = true;
  // argv[2]: a comma-separated list of kinds to run (default: all)
  const std::string only = argc > 2 ? std::string(",") + argv[2] + "," : "";
  for (int k = 0; k < NKIND; k++) {
    if (!only.empty() && only.find(std::string(",") + kKindName[k] + ",") == std::string::npos)
      continue;
    KFn fn = kernel_of(k);
    for (int w : wps) {
      const size_t lds = lds_cu / (4 * w) - 256;  // <= 4 W one-wave workgroups per CU
      CHECK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      const int blocks = cus * 4 * w * gens;
      hipLaunchKernelGGL(fn, dim3(blocks), dim3(64), lds, 0, out, cyc, iters / 8);  // warm
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(fn, dim3(blocks), dim3(64), lds, 0, out, cyc, iters);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      CHECK(hipMemcpy(hc.data(), cyc, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      double cyc_sum = 0;
      for (int b = 0; b < blocks; b++) cyc_sum += (double)hc[b];
      const double cyc_wave = cyc_sum / blocks;
      const double valu_wave = (double)kValuPerIter[k] * iters;
      const double valu = valu_wave * blocks;
      const double rate_simd = valu / (ms * 1e-3) / simds;  // wave-instructions / s / SIMD
      // SIMD cycles per VALU instruction at the nominal clock (prop.clockRate), from the launch
      // time. (The per-wave s_memtime span is reported as measured; it does not give cycles per
      // instruction, as waves are not all co-resident from start to end: r04_run2 implied clocks
      // of 0.8-2.4 GHz for one launch configuration.)
      const double cpi_nominal = prop.clockRate * 1e3 / rate_simd;
      printf("%s{\"kind\": \"%s\", \"waves_per_simd\": %d, \"valu_per_wave\": %.0f, \"salu_per_wave\": %.0f, "
             "\"ms\": %.4f, \"g_valu_per_s_chip\": %.2f, \"g_valu_per_s_simd\": %.5f, "
             "\"cycles_per_valu_simd_nominal\": %.4f, \"smemtime_cycles_per_wave\": %.0f}",
             first ? "" : ", ", kKindName[k], w, valu_wave, (double)kSaluPerIter[k] * iters, ms,
             valu / (ms * 1e-3) / 1e9, rate_simd / 1e9, cpi_nominal, cyc_wave);
      first = false;
      fflush(stdout);
    }
  }
  printf("]}\n");
  CHECK(hipFree(out));
  CHECK(hipFree(cyc));
  return 0;
}
