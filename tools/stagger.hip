// stagger.hip — hold every wave slot of the GPU, then free the slots one by one (debugging aid
// for the wrong-result variants, DESIGN.md § Wrong-result variants).
//
// The failing c3 variant fails mostly in the first generation of its waves, when every CU's 16
// slots fill at once. A launch queued behind this kernel on another stream gets its slots in the
// order this kernel frees them: with `spread_ms` > 0 its first generation starts staggered over
// that time, at the same occupancy once every slot is free; `spread_ms` 0 frees them together.
//
// A wave allocates what one analyze wave of the variant does (128 VGPRs, 6,464 B of LDS, one wave
// per workgroup), so one wave per slot: 4 per SIMD, 16 per CU, 4,096 on the chip. Each spins on
// the 100 MHz wall clock until start_ms + spread_ms * (its block index / waves) after its own start.
//
//   hipcc -shared -fPIC --offload-arch=gfx950 -O3 -o build/bin/libstagger.so tools/stagger.hip
//   lt_stagger(waves, start_ms, spread_ms) -> 0 or a hipError_t (launched on a non-blocking stream
//   of its own, returns at once); lt_hold(waves, ms, big) / lt_hold_ids (below)
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(64, 4) void stagger_kernel(uint64_t start_ticks, uint64_t spread_ticks,
                                                        unsigned waves, uint32_t* sink) {
  __shared__ uint32_t pad[6464 / 4];
  pad[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const uint64_t t0 = wall_clock64();
  const uint64_t until = t0 + start_ticks + spread_ticks * blockIdx.x / waves;
  uint32_t acc = pad[(threadIdx.x + 1) & 63];
  while (wall_clock64() < until) acc += 1;
  // the allocation of a variant wave: v0-v127 named as clobbered
  asm volatile("" ::: "v127");
  if (acc == 0xffffffffu) sink[threadIdx.x] = acc;  // never true in practice; keeps the loop
}

// hold: WAVES waves that keep their slots for `ms` after their own start, each recording where it
// runs (HW_ID: wave, SIMD, CU, SE; XCC_ID), so a launch queued behind it runs beside them at the
// occupancy they leave. BIG: a wave of the variant's size (128 VGPRs, 6,464 B of LDS); else a
// small one (a few VGPRs, no LDS) that takes a wave slot but little of the register file.
template <bool BIG>
__global__ __launch_bounds__(64, BIG ? 4 : 8) void hold_kernel(uint64_t ticks, uint32_t* ids) {
  uint32_t acc = 0;
  if constexpr (BIG) {
    __shared__ uint32_t pad[6464 / 4];
    pad[threadIdx.x] = threadIdx.x;
    __syncthreads();
    acc = pad[(threadIdx.x + 1) & 63];
  }
  const uint64_t until = wall_clock64() + ticks;
  while (wall_clock64() < until) acc += 1;
  if constexpr (BIG) asm volatile("" ::: "v127");
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
  const uint32_t xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // XCC_ID
  if (threadIdx.x == 0) {
    ids[2 * blockIdx.x] = hw;
    ids[2 * blockIdx.x + 1] = xcc;
  }
  if (acc == 0xffffffffu) ids[0] = acc;  // never true in practice; keeps the loop
}

static hipStream_t g_stream = nullptr;
static uint32_t* g_ids = nullptr;
static int g_ids_n = 0;
static uint32_t* g_sink = nullptr;

extern "C" int lt_stagger(int waves, double start_ms, double spread_ms) {
  if (!g_stream) {
    hipError_t e = hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking);
    if (e != hipSuccess) return (int)e;
    e = hipMalloc(&g_sink, 64 * sizeof(uint32_t));
    if (e != hipSuccess) return (int)e;
  }
  const uint64_t tps = 100000;  // wall clock ticks per ms (100 MHz)
  hipLaunchKernelGGL(stagger_kernel, dim3(waves), dim3(64), 0, g_stream,
                     (uint64_t)(start_ms * tps), (uint64_t)(spread_ms * tps), (unsigned)waves,
                     g_sink);
  return (int)hipGetLastError();
}

extern "C" int lt_hold(int waves, double ms, int big) {
  if (!g_stream) {
    hipError_t e = hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking);
    if (e != hipSuccess) return (int)e;
  }
  if (g_ids_n < waves) {
    if (g_ids) (void)hipFree(g_ids);
    hipError_t e = hipMalloc(&g_ids, 2 * sizeof(uint32_t) * waves);
    if (e != hipSuccess) return (int)e;
    g_ids_n = waves;
  }
  const uint64_t ticks = (uint64_t)(ms * 100000);
  if (big)
    hipLaunchKernelGGL(hold_kernel<true>, dim3(waves), dim3(64), 0, g_stream, ticks, g_ids);
  else
    hipLaunchKernelGGL(hold_kernel<false>, dim3(waves), dim3(64), 0, g_stream, ticks, g_ids);
  return (int)hipGetLastError();
}

// after lt_stagger_wait(): the (HW_ID, XCC_ID) pair of each hold wave
extern "C" int lt_hold_ids(uint32_t* out, int waves) {
  if (waves > g_ids_n) return -1;
  return (int)hipMemcpy(out, g_ids, 2 * sizeof(uint32_t) * waves, hipMemcpyDeviceToHost);
}

extern "C" int lt_stagger_wait() { return g_stream ? (int)hipStreamSynchronize(g_stream) : 0; }
