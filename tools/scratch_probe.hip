// scratch_probe.hip — does every resident wave get private (scratch) memory of its own?
// (debugging aid for the wrong-result JIT variants, DESIGN.md § Wrong-result variants.)
//
// Each lane fills a dynamically indexed private array (kept in scratch, like the analyze
// kernel's OPTa / AG arrays and its spill slots) with a pattern of its global wave id, lane and
// slot, spins for a while (so many waves are resident at once), then reads every slot back and
// counts the slots that do not hold its own pattern. A kernel whose waves shared scratch (or
// read a neighbour's) would count mismatches. Two register budgets: a light kernel (8 waves per
// SIMD) and one held at 128 VGPRs by launch bounds and live values (4 waves per SIMD, the
// analyze kernel's occupancy). Prints one JSON object.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#ifndef PROBE_SLOTS
#define PROBE_SLOTS 80  // 320 B per lane, the LT_PASSB_SLOTS=0 c3 instance's private segment
#endif

struct Bad {
  unsigned long long count;
  unsigned long long first;  // wave << 16 | lane << 8 | slot of one mismatch
  unsigned int got, want;
};

__device__ inline unsigned pattern(unsigned long long wave, int lane, int slot) {
  return (unsigned)(wave * 2654435761ull) ^ ((unsigned)lane << 24) ^ ((unsigned)slot * 40503u);
}

template <int HEAVY>
__device__ void probe(Bad* bad, int spin, int salt) {
  unsigned priv[PROBE_SLOTS];  // per-lane dynamic indices: the array stays in scratch
  const int lane = threadIdx.x & 63;
  const unsigned long long wave = (unsigned long long)blockIdx.x * (blockDim.x >> 6) +
                                  (threadIdx.x >> 6);
  for (int i = 0; i < PROBE_SLOTS; i++) priv[(i * 7 + lane) % PROBE_SLOTS] =
      pattern(wave, lane, (i * 7 + lane) % PROBE_SLOTS);
  __asm__ __volatile__("" ::: "memory");  // no store-to-load forwarding across the spin
  // work in registers while the array sits in scratch: HEAVY keeps ~100 values live
  double acc[HEAVY ? 58 : 1];
#pragma unroll
  for (int k = 0; k < (HEAVY ? 58 : 1); k++) acc[k] = (double)(lane + k + salt);
  for (int s = 0; s < spin; s++) {
#pragma unroll
    for (int k = 0; k < (HEAVY ? 58 : 1); k++) acc[k] = __builtin_fma(acc[k], 1.0000001, 1e-9);
  }
  double sum = 0.0;
#pragma unroll
  for (int k = 0; k < (HEAVY ? 58 : 1); k++) sum += acc[k];
  __asm__ __volatile__("" ::: "memory");
  unsigned nbad = 0, g = 0, w = 0;
  int slot = -1;
  for (int i = 0; i < PROBE_SLOTS; i++) {
    const int j = (i * 13 + lane + salt) % PROBE_SLOTS;
    const unsigned v = priv[j], e = pattern(wave, lane, j);
    if (v != e) {
      nbad++;
      slot = j;
      g = v;
      w = e;
    }
  }
  if (sum == -1.0) nbad += 1000000;  // keeps the register work live
  if (nbad) {
    atomicAdd(&bad->count, (unsigned long long)nbad);
    atomicExch(&bad->first, (wave << 16) | ((unsigned long long)lane << 8) | (unsigned)slot);
    atomicExch(&bad->got, g);
    atomicExch(&bad->want, w);
  }
}

__global__ __launch_bounds__(64) void probe_light(Bad* bad, int spin, int salt) {
  probe<0>(bad, spin, salt);
}
__global__ __launch_bounds__(64, 4) void probe_heavy(Bad* bad, int spin, int salt) {
  probe<1>(bad, spin, salt);
}

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                       \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

int main(int argc, char** argv) {
  const int waves = argc > 1 ? atoi(argv[1]) : 1 << 20;
  const int spin = argc > 2 ? atoi(argv[2]) : 200;
  const int reps = argc > 3 ? atoi(argv[3]) : 4;
  Bad* d;
  CK(hipMalloc(&d, sizeof(Bad)));
  printf("{\"slots\": %d, \"waves\": %d, \"spin\": %d, \"runs\": [", PROBE_SLOTS, waves, spin);
  for (int r = 0; r < 2 * reps; r++) {
    const bool heavy = r & 1;
    CK(hipMemset(d, 0, sizeof(Bad)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    if (heavy) hipLaunchKernelGGL(probe_heavy, dim3(waves), dim3(64), 0, 0, d, spin, r);
    else hipLaunchKernelGGL(probe_light, dim3(waves), dim3(64), 0, 0, d, spin, r);
    CK(hipGetLastError());
    CK(hipEventRecord(b));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    Bad h;
    CK(hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost));
    printf("%s{\"kernel\": \"%s\", \"ms\": %.3f, \"mismatched_slots\": %llu, \"first\": [%llu, %llu, "
           "%llu], \"got\": %u, \"want\": %u}",
           r ? ", " : "", heavy ? "heavy_128vgpr" : "light", ms, h.count, h.first >> 16,
           (h.first >> 8) & 255, h.first & 255, h.got, h.want);
  }
  printf("]}\n");
  return 0;
}
