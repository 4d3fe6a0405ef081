// lt_abi.hip — the C ABI of include/lt_abi.h: contexts, argument checks, scene upload, launches.
//
// Replaces, per pixel tile, the per-grid-point loop of MRLandTrendrJob.analysis_reducer
// (/root/reference/mr_land_trendr_job.py:83-126) around utils.analyze + utils.change_labeling.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lt_abi.h"
#include "lt_launch.h"
#include "lt_pixel.h"
#include "lt_index.h"
#include "lt_jit.h"
#include "lt_kernels_dev.h"
#include "lt_settings.h"
#include "lt_raster.h"

namespace {

constexpr int kBlock = 256;

// one lsq_factor per slot of the x-set table (lt_lapack.h), computed by the device arithmetic
// that the lookups replace
__global__ __launch_bounds__(kBlock) void build_xtable_kernel(lt::lsq_xf* __restrict__ xtab) {
  const int idx = blockIdx.x * kBlock + threadIdx.x;
  if (idx >= lt::kXtSize) return;
  int m = 0, xs[64];
  lt::lsq_xf f{};
  if (lt::xset_of_key(idx, m, xs))
    lt::lsq_factor(m, [&](int k) { return xs[k]; }, f);
  else
    f.rc = -4;  // no x-set maps here
  xtab[idx] = f;
}

// The spike / vertex planes from the per-pixel year flags the analyze and resolve stages leave
// (lt_fast.h): four pixels per thread, so each year row of a wave is one 256-byte store per plane
// (a wave of the analyze kernel would write 64-byte pieces, which cost far more than their bytes).
// V4: the planes and their stride are 4-byte aligned (else one pixel per thread).
template <bool V4>
__global__ __launch_bounds__(kBlock) void year_flags_kernel(const uint64_t* __restrict__ yflags,
                                                            int64_t n, int Y,
                                                            uint8_t* __restrict__ spike,
                                                            uint8_t* __restrict__ vertex,
                                                            int64_t os) {
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if constexpr (V4) {
    const int64_t p = t * 4;
    if (p >= n) return;
    const int np = n - p < 4 ? (int)(n - p) : 4;
    uint64_t sf[4] = {0, 0, 0, 0}, vf[4] = {0, 0, 0, 0};
    for (int i = 0; i < np; i++) {
      sf[i] = yflags[p + i];
      vf[i] = yflags[n + p + i];
    }
    for (int y = 0; y < Y; y++) {
      uint32_t a = 0, b = 0;
      for (int i = 0; i < 4; i++) {
        a |= (uint32_t)((sf[i] >> y) & 1) << (8 * i);
        b |= (uint32_t)((vf[i] >> y) & 1) << (8 * i);
      }
      const int64_t o = (int64_t)y * os + p;
      if (np == 4) {
        if (spike) __builtin_nontemporal_store(a, (uint32_t*)(spike + o));
        if (vertex) __builtin_nontemporal_store(b, (uint32_t*)(vertex + o));
      } else {
        for (int i = 0; i < np; i++) {
          if (spike) spike[o + i] = (uint8_t)(a >> (8 * i));
          if (vertex) vertex[o + i] = (uint8_t)(b >> (8 * i));
        }
      }
    }
  } else {
    if (t >= n) return;
    const uint64_t sf = yflags[t], vf = yflags[n + t];
    for (int y = 0; y < Y; y++) {
      const int64_t o = (int64_t)y * os + t;
      if (spike) spike[o] = (uint8_t)((sf >> y) & 1);
      if (vertex) vertex[o] = (uint8_t)((vf >> y) & 1);
    }
  }
}

// The per-year trendline planes from the compact trendline the analyze / resolve stages leave
// (lt_fast.h tl_split): eqns2fitted_points (utils.py:682-722) and the TrendlinePoint fields
// (classes.py:67-116). Everything follows from the pixel's four words — present years P0 (0: the
// reference raises), spike flags by present index, vertices by non-spike index, the left-eqn
// choice by vertex number — and the segment eqns:
//   t = present index of slot y, spike = bit t, k = its non-spike index, vertex = bit k;
//   passed = vertices at or before the point; the current eqn is segment passed-1, or, past the
//   last vertex (whose eqn is its left segment's, utils.py:662), segment n_vertices-2;
//   val_fit = m x + b of the current eqn (x = year offset from the first present year, no FMA),
//   or of the previous one at an interior vertex that took the left eqn;
//   fit_m / fit_b = the eqn used, right_m / right_b = the current one; NaN for absent years.
// Exactly the values of the year-major loop (lt_fast.h, tl_split off), which it replaces.
// One thread per (pixel, chunk of kYC year slots): its four words, then every eqn the chunk's
// years use (all loads in flight together), then the chunk's rows (stores only: no store before
// a load in a thread). A thread per (pixel, year) waited out three dependent load round trips per
// seven stores: 9.3 ms per 16.8 Mpx c5 tile, 3.0 TB/s (profiles/r05_run5). Blocks: 256 pixels of
// one chunk, the chunks of a pixel range consecutive (its words and eqns then come from L2).
constexpr int kYC = 8;
__global__ __launch_bounds__(kBlock) void trendline_expand_kernel(
    const lt::DevScene* __restrict__ S, const uint64_t* __restrict__ bits,
    const double* __restrict__ eqn, int64_t n, int Y, const lt_tile_out out) {
  const int nch = (Y + kYC - 1) / kYC;
  const int ya = (int)(blockIdx.x % (unsigned)nch) * kYC;
  const int64_t p = (int64_t)(blockIdx.x / (unsigned)nch) * kBlock + threadIdx.x;
  if (p >= n) return;
  const uint64_t P0 = bits[p], SP = bits[n + p], VM = bits[2 * n + p], LB = bits[3 * n + p];
  const int nvt = __builtin_popcountll(VM);
  typedef double d2 __attribute__((ext_vector_type(2)));
  d2 cur[kYC], prv[kYC];
  // (1) every eqn the chunk needs, loads issued together
#pragma unroll
  for (int j = 0; j < kYC; j++) {
    const int y = ya + j;
    cur[j] = d2{0.0, 0.0};
    prv[j] = d2{0.0, 0.0};
    if (y >= Y || !((P0 >> y) & 1)) continue;
    const int t = __builtin_popcountll(P0 & ((1ull << y) - 1));  // y <= 63
    const bool sp = (SP >> t) & 1;
    const int k = t - __builtin_popcountll(SP & ((1ull << t) - 1));
    const bool vx = !sp && ((VM >> k) & 1);
    const uint64_t upto = sp ? ((1ull << k) - 1) : (k >= 63 ? ~0ull : ((2ull << k) - 1));
    const int qc = __builtin_popcountll(VM & upto) - 1;  // the last vertex at or before the point
    const int e = qc + 1 >= nvt ? nvt - 2 : qc;
    if (e >= 0) cur[j] = *(const d2*)(eqn + 2 * ((int64_t)e * n + p));
    if (vx && qc > 0 && qc < nvt - 1 && ((LB >> qc) & 1))
      prv[j] = *(const d2*)(eqn + 2 * ((int64_t)(qc - 1) * n + p));
  }
  // (2) the rows
  const double nan = __builtin_nan("");
  const int32_t y0 = P0 ? S->year[__builtin_ctzll(P0)] : 0;
#pragma unroll
  for (int j = 0; j < kYC; j++) {
    const int y = ya + j;
    if (y >= Y) break;
    double fv = nan, fm = nan, fb = nan, rm = nan, rb = nan;
    uint8_t sp = 0, vx = 0;
    if ((P0 >> y) & 1) {
      const int t = __builtin_popcountll(P0 & ((1ull << y) - 1));
      sp = (uint8_t)((SP >> t) & 1);
      const int k = t - __builtin_popcountll(SP & ((1ull << t) - 1));
      vx = (uint8_t)(!sp && ((VM >> k) & 1));
      const uint64_t upto = sp ? ((1ull << k) - 1) : (k >= 63 ? ~0ull : ((2ull << k) - 1));
      const int qc = __builtin_popcountll(VM & upto) - 1;
      const double x = (double)(S->year[y] - y0);
      rm = cur[j].x;
      rb = cur[j].y;
      const bool lft = vx && qc > 0 && qc < nvt - 1 && ((LB >> qc) & 1);
      fm = lft ? prv[j].x : rm;
      fb = lft ? prv[j].y : rb;
      fv = (fm * x) + fb;
    }
    const int64_t o = (int64_t)y * out.stride + p;
    if (out.val_fit) __builtin_nontemporal_store(fv, out.val_fit + o);
    if (out.fit_m) __builtin_nontemporal_store(fm, out.fit_m + o);
    if (out.fit_b) __builtin_nontemporal_store(fb, out.fit_b + o);
    if (out.right_m) __builtin_nontemporal_store(rm, out.right_m + o);
    if (out.right_b) __builtin_nontemporal_store(rb, out.right_b + o);
    if (out.spike) out.spike[o] = sp;
    if (out.vertex) out.vertex[o] = vx;
  }
}

struct YearArg {
  int32_t year[LT_MAX_YEARS];
};

__global__ __launch_bounds__(kBlock) void label_kernel(const YearArg yrs, int Y, const lt_params P,
                                                       const lt_label_in in,
                                                       const lt_tile_out out) {
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= in.n_pix) return;
  lt::label_pixel(yrs.year, Y, P, in, out, p);
}

struct EventPair {
  hipEvent_t start, stop;
};

// output raster assembly (lt_raster.h): fill every raster pixel, then scatter the selected grid
// points; with identity offsets one pass writes both. Grid-stride, coalesced in the pixel index.
__global__ __launch_bounds__(kBlock) void raster_fill_kernel(const lt_raster_job J) {
  const double nodata = J.mode == LT_RASTER_REFERENCE ? (double)LT_NODATA : J.fill;
  for (int64_t o = (int64_t)blockIdx.x * kBlock + threadIdx.x; o < J.n_out;
       o += (int64_t)gridDim.x * kBlock)
    lt::raster_store(J, o, nodata);
}

// presence bitmap of winning obs ids: per block in LDS, then one global OR per word
__global__ __launch_bounds__(kBlock) void winner_presence_kernel(const int16_t* __restrict__ w,
                                                                 int64_t stride, int Y,
                                                                 int64_t n_pix, int n_obs,
                                                                 uint32_t* __restrict__ bits) {
  __shared__ uint32_t loc[LT_MAX_OBS / 32];
  const int nw = (n_obs + 31) / 32;
  for (int k = threadIdx.x; k < nw; k += kBlock) loc[k] = 0u;
  __syncthreads();
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < n_pix;
       p += (int64_t)gridDim.x * kBlock)
    for (int y = 0; y < Y; y++) {
      const int o = w[(int64_t)y * stride + p];
      if (o >= 0 && o < n_obs) atomicOr(&loc[o >> 5], 1u << (o & 31));
    }
  __syncthreads();
  for (int k = threadIdx.x; k < nw; k += kBlock)
    if (loc[k]) atomicOr(&bits[k], loc[k]);
}

__global__ __launch_bounds__(kBlock) void raster_scatter_kernel(const lt_raster_job J,
                                                                bool fill_too) {
  const double nodata = J.mode == LT_RASTER_REFERENCE ? (double)LT_NODATA : J.fill;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < J.n_pix;
       p += (int64_t)gridDim.x * kBlock) {
    const bool sel = lt::raster_selected(J, p);
    if (!sel && !fill_too) continue;
    const double v = !sel ? nodata
                          : (J.plane ? lt::plane_value(J.plane, J.plane_type, p) : J.const_value);
    lt::raster_store(J, J.dest ? J.dest[p] : p, v);
  }
}

}  // namespace

// One JIT module of the context (lt_jit.h): compiled on the launching thread (LT_JIT_SYNC) or on
// a worker (LT_JIT_ASYNC, lt_jit_prepare without wait), loaded on the launching thread once done.
struct JitJob {
  std::string src, arch, code, err;
  bool ok = false, disk_hit = false;
  std::atomic<bool> done{false};
};
struct JitEntry {
  int state = 0;  // 0 compiling, 1 ready, -1 failed (its tiles take the precompiled kernels)
  lt_jit_kernels k;
  bool has_r64 = false, scene_spec = false;
  std::string err;
  std::shared_ptr<JitJob> job;
  std::thread worker;
  uint64_t last_use = 0;
  hipEvent_t ev_last = nullptr;  // after the last resolve launch that used the module
};

struct lt_ctx {
  int device = 0;
  std::string err;
  lt::DevScene* h_scene = nullptr;  // pinned staging
  lt::DevScene* d_scene = nullptr;
  hipEvent_t scene_copied = nullptr;
  bool scene_valid = false;
  bool timing = false;
  std::vector<EventPair> pool;   // all events ever created (reused): 2 pairs per launch
  size_t used = 0;               // pairs recorded since the last stage_ms call
  int64_t launches = 0;
  int64_t* d_defer = nullptr;    // deferred-pixel list of the resolve stage
  uint64_t* d_yflags = nullptr;  // per-pixel spike / vertex year flags (kSets sets x 2 planes)
  unsigned long long* d_ndefer = nullptr;
  int64_t defer_cap = 0;
  lt::lsq_xf* d_xtab = nullptr;  // x-set factor table (built at context creation)
  hipStream_t side = nullptr;    // the resolve stage's stream (lt_analyze_tiles)
  // deferred-list sets, used round robin by consecutive tiles (also across calls): tile t's
  // set is reused by tile t + n_sets only after tile t's resolve
  static constexpr int kSets = 3;
  int n_sets = kSets;  // LT_DEFER_SETS (2..3) for A/B runs
  hipEvent_t ev_analyzed[kSets] = {};
  hipEvent_t ev_resolved[kSets] = {};
  bool set_used[kSets] = {};
  int last_set = 0, next_set = 0;
  std::map<std::string, lt_index*> index_fns;  // compiled load-stage kernels, by source
  // JIT analyze / resolve kernels with an index_eqn program inlined (lt_jit.h), by spec_key
  std::map<uint64_t, JitEntry> jit;
  int jit_mode = LT_JIT_SYNC;
  uint64_t jit_clock = 0;      // launch counter for the modules' least-recently-used order
  int jit_max_modules = 16;    // LT_JIT_MAX_MODULES
  int jit_scene_max = 8;       // LT_JIT_SCENE_MAX: scene-specialised modules before the generic
  lt_jit_stats jstats{};
  std::string jit_err;         // the last JIT failure
  std::string arch;            // the device's target id (hiprtc --offload-arch)
  // the precompiled fallback of a non-linear program: its index raster per deferred-list set
  void* d_iscratch[kSets] = {};
  size_t iscratch_bytes[kSets] = {};
  // the compact trendline per deferred-list set (lt_fast.h tl_split): [4][cap] words and
  // [Y-1][cap] segment eqns, written by analyze / resolve, read by trendline_expand_kernel
  uint64_t* d_tl_bits[kSets] = {};
  double* d_tl_eqn[kSets] = {};
  int64_t tl_cap[kSets] = {};
  int tl_segs[kSets] = {};
  hipStream_t xstream = nullptr;  // the expand kernel's stream (LT_EXPAND_PRIORITY)
  hipEvent_t ev_rdone[kSets] = {};  // a tile's resolve kernels done (the expand kernel waits)
  hipEvent_t ev_xdone = nullptr;    // the last expand kernel queued
  bool x_used = false;
  hipStream_t last_stage = nullptr;  // the stream of the last tile's last stage
  // LT_TL_SPLIT=1 at creation: per-year planes through the compact trendline and the expand
  // kernel. Off by default: measured slower on c5 (899 vs 1228 Mpx/s, profiles/r05_run6): the
  // analyze kernel drops from 12.3 to 9.0-9.3 ms per 16.8 Mpx tile, but the expand kernel takes
  // 8.1 ms alone (28 GB of rows at 3.5 TB/s) and gets CU slots only between analyze launches
  bool tl_split = false;
};

static int fail(lt_ctx* c, int code, const char* fmt, const char* detail = "") {
  if (c) {
    char buf[512];
    snprintf(buf, sizeof buf, fmt, detail);
    c->err = buf;
  }
  return code;
}

#define HIP_OR_FAIL(ctx, expr)                                       \
  do {                                                               \
    hipError_t e_ = (expr);                                          \
    if (e_ != hipSuccess) return fail(ctx, LT_ERR_HIP, #expr ": %s", \
                                      hipGetErrorString(e_));        \
  } while (0)

extern "C" {

int lt_abi_version(void) { return LT_ABI_VERSION; }

int lt_settings_compile(const char* settings_json, int32_t pre_threshold_mode, int32_t band_type,
                        int32_t out_type, int32_t raster_count, lt_settings* out,
                        int32_t* exc_kind, char* err, int64_t err_cap) {
  if (exc_kind) *exc_kind = LT_EXC_NONE;
  if (err && err_cap > 0) err[0] = 0;
  try {
    lt_set::compile(settings_json, pre_threshold_mode, band_type, out_type, raster_count, out);
    return LT_OK;
  } catch (const lt_set::Fail& f) {
    if (exc_kind) *exc_kind = f.exc;
    if (err && err_cap > 0) {
      const size_t n = f.msg.size() < (size_t)(err_cap - 1) ? f.msg.size() : (size_t)(err_cap - 1);
      memcpy(err, f.msg.data(), n);
      err[n] = 0;
    }
    return f.code;
  } catch (...) {
    if (exc_kind) *exc_kind = LT_EXC_OTHER;
    return LT_ERR_ARG;
  }
}

int lt_ctx_create(int device, lt_ctx** out) {
  if (!out) return LT_ERR_ARG;
  *out = nullptr;
  lt_ctx* c = new lt_ctx();
  c->device = device;
  // JIT module cache bounds (lt_abi.h LT_JIT_*; tests and long-running mosaics)
  if (const char* e = getenv("LT_JIT_MAX_MODULES"))
    if (atoi(e) >= 1) c->jit_max_modules = atoi(e);
  if (const char* e = getenv("LT_JIT_SCENE_MAX"))
    if (atoi(e) >= 0) c->jit_scene_max = atoi(e);
  if (const char* e = getenv("LT_TL_SPLIT")) c->tl_split = e[0] == '1';
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipHostMalloc((void**)&c->h_scene, sizeof(lt::DevScene));
  if (e == hipSuccess) e = hipMalloc((void**)&c->d_scene, sizeof(lt::DevScene));
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->scene_copied, hipEventDisableTiming);
  if (e == hipSuccess) e = hipMalloc((void**)&c->d_xtab, sizeof(lt::lsq_xf) * lt::kXtSize);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(build_xtable_kernel, dim3((lt::kXtSize + kBlock - 1) / kBlock),
                       dim3(kBlock), 0, 0, c->d_xtab);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    lt_ctx_destroy(c);
    return LT_ERR_HIP;
  }
  *out = c;
  return LT_OK;
}

int lt_ctx_destroy(lt_ctx* c) {
  if (!c) return LT_OK;
  (void)hipSetDevice(c->device);
  if (c->scene_copied) {
    (void)hipEventSynchronize(c->scene_copied);
    (void)hipEventDestroy(c->scene_copied);
  }
  for (auto& ep : c->pool) {
    (void)hipEventDestroy(ep.start);
    (void)hipEventDestroy(ep.stop);
  }
  if (c->side) {
    (void)hipStreamSynchronize(c->side);
    (void)hipStreamDestroy(c->side);
  }
  for (int s = 0; s < lt_ctx::kSets; s++) {
    if (c->ev_analyzed[s]) (void)hipEventDestroy(c->ev_analyzed[s]);
    if (c->ev_resolved[s]) (void)hipEventDestroy(c->ev_resolved[s]);
  }
  for (auto& kv : c->jit) {
    if (kv.second.worker.joinable()) kv.second.worker.join();
    if (kv.second.ev_last) (void)hipEventDestroy(kv.second.ev_last);
    if (kv.second.k.mod) (void)hipModuleUnload(kv.second.k.mod);
  }
  if (c->xstream) {
    (void)hipStreamSynchronize(c->xstream);
    (void)hipStreamDestroy(c->xstream);
  }
  if (c->ev_xdone) (void)hipEventDestroy(c->ev_xdone);
  for (int s = 0; s < lt_ctx::kSets; s++) {
    if (c->d_iscratch[s]) (void)hipFree(c->d_iscratch[s]);
    if (c->d_tl_bits[s]) (void)hipFree(c->d_tl_bits[s]);
    if (c->d_tl_eqn[s]) (void)hipFree(c->d_tl_eqn[s]);
    if (c->ev_rdone[s]) (void)hipEventDestroy(c->ev_rdone[s]);
  }
  if (c->d_defer) (void)hipFree(c->d_defer);
  if (c->d_yflags) (void)hipFree(c->d_yflags);
  if (c->d_ndefer) (void)hipFree(c->d_ndefer);
  if (c->d_scene) (void)hipFree(c->d_scene);
  if (c->d_xtab) (void)hipFree(c->d_xtab);
  for (auto& kv : c->index_fns) {
    if (kv.second->mod) (void)hipModuleUnload(kv.second->mod);
    delete kv.second;
  }
  if (c->h_scene) (void)hipHostFree(c->h_scene);
  delete c;
  return LT_OK;
}

const char* lt_last_error(const lt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int lt_ctx_set_timing(lt_ctx* c, int enable) {
  if (!c) return LT_ERR_ARG;
  c->timing = enable != 0;
  return LT_OK;
}

int lt_ctx_stage_ms(lt_ctx* c, double* ms_out, int n_stages, int64_t* n_launches) {
  if (!c) return LT_ERR_ARG;
  HIP_OR_FAIL(c, hipSetDevice(c->device));
  double acc[3] = {0.0, 0.0, 0.0};
  for (size_t i = 0; i < c->used; i++) {
    HIP_OR_FAIL(c, hipEventSynchronize(c->pool[i].stop));
    float ms = 0.f;
    HIP_OR_FAIL(c, hipEventElapsedTime(&ms, c->pool[i].start, c->pool[i].stop));
    acc[i % 3] += ms;  // pairs cycle: analyze stage, resolve stage, trendline expand
  }
  for (int s = 0; s < n_stages; s++) ms_out[s] = s < 3 ? acc[s] : 0.0;
  if (n_launches) *n_launches = c->launches;
  c->used = 0;
  c->launches = 0;
  return LT_OK;
}

static int check_tile(lt_ctx* c, const lt_tile_in* in, const lt_tile_out* out) {
  if (!in || !out) return fail(c, LT_ERR_ARG, "null argument%s");
  if (in->n_pix < 0 || in->stride < in->n_pix || out->stride < in->n_pix)
    return fail(c, LT_ERR_ARG, "bad n_pix/stride%s");
  if (in->n_pix > LT_MAX_TILE_PIX) return fail(c, LT_ERR_LIMIT, "tile above LT_MAX_TILE_PIX%s");
  if (in->n_pix == 0) return LT_OK;  // nothing is read or written
  if (in->obs_bands && in->index) {  // the fused load stage, any program (JIT kernels)
    const lt_index* f = in->index;
    const bool planar = in->band_pix_stride == 1 && in->band_stride >= in->n_pix &&
                        in->band_obs_stride >= (int64_t)f->n_bands * in->band_stride;
    const bool interleaved = in->band_stride == 1 && in->band_pix_stride == f->n_bands &&
                             in->band_obs_stride >= (int64_t)f->n_bands * in->n_pix;
    if (!planar && !interleaved) return fail(c, LT_ERR_ARG, "bad band strides%s");
    return LT_OK;
  }
  if (in->obs_bands) {  // the fused load stage: a linear form lt_index_linearize accepts
    const lt_index_lin& L = in->lin;
    if (L.n_bands < 1 || L.n_bands > LT_LIN_MAX_BANDS ||
        (L.band_type != LT_T_I16 && L.band_type != LT_T_U16 && L.band_type != LT_T_U8 &&
         L.band_type != LT_T_I32) ||
        !lt_idx::is_int(L.wrap_type) || !lt_idx::ctype(L.out_type))
      return fail(c, LT_ERR_ARG, "bad linear index form%s");
    const bool planar = in->band_pix_stride == 1 && in->band_stride >= in->n_pix &&
                        in->band_obs_stride >= (int64_t)L.n_bands * in->band_stride;
    const bool interleaved = in->band_stride == 1 && in->band_pix_stride == L.n_bands &&
                             in->band_obs_stride >= (int64_t)L.n_bands * in->n_pix;
    if (!planar && !interleaved) return fail(c, LT_ERR_ARG, "bad band strides%s");
    const int64_t esz = (int64_t)lt_idx::type_size(L.band_type);
    if (interleaved && L.n_bands == 2 && esz == 2 &&
        ((uintptr_t)in->obs_bands % 4 != 0 || in->band_obs_stride % 2 != 0))
      return fail(c, LT_ERR_ARG, "interleaved int16 band pairs must be 4-byte aligned%s");
    return LT_OK;
  }
  if (!in->obs_val && !in->obs_index) return fail(c, LT_ERR_ARG, "obs_val or obs_index required%s");
  if (in->obs_index && !lt_idx::ctype(in->index_type))
    return fail(c, LT_ERR_ARG, "bad index_type%s");
  return LT_OK;
}

// Per-year planes with the compact trendline (lt_fast.h tl_split, trendline_expand_kernel):
// every launch asking for any of them when the context was created with LT_TL_SPLIT=1 (else the
// year-major loop writes them)
static bool tl_split_launch(const lt_ctx* c, const lt_tile_out* o) {
  return c->tl_split && (o->val_fit || o->fit_m || o->fit_b || o->right_m || o->right_b ||
                         o->spike || o->vertex);
}

// the device's target id, for hiprtc (cached)
static int device_arch(lt_ctx* c) {
  if (!c->arch.empty()) return LT_OK;
  hipDeviceProp_t prop;
  HIP_OR_FAIL(c, hipGetDeviceProperties(&prop, c->device));
  c->arch = prop.gcnArchName;
  return LT_OK;
}

// Unload least-recently-used ready modules past the cap (LT_JIT_MAX_MODULES), never `keep`: a
// module's last resolve launch is waited for first, so no queued kernel loses its code
static void jit_evict(lt_ctx* c, uint64_t keep) {
  for (;;) {
    int ready = 0;
    auto lru = c->jit.end();
    for (auto it = c->jit.begin(); it != c->jit.end(); ++it) {
      if (it->second.state != 1) continue;
      ready++;
      if (it->first != keep && (lru == c->jit.end() || it->second.last_use < lru->second.last_use))
        lru = it;
    }
    if (ready <= c->jit_max_modules || lru == c->jit.end()) return;
    JitEntry& e = lru->second;
    if (e.ev_last) {
      (void)hipEventSynchronize(e.ev_last);
      (void)hipEventDestroy(e.ev_last);
    }
    if (e.k.mod) (void)hipModuleUnload(e.k.mod);
    c->jit.erase(lru);
    c->jstats.evictions++;
  }
}

// A compiling entry whose job is done (or, when `wait`, once it is): join the worker, load the
// module on this thread, count it
static void jit_finish(lt_ctx* c, uint64_t key, JitEntry& e, bool wait) {
  if (e.state != 0) return;
  if (!e.job->done.load(std::memory_order_acquire)) {
    if (!wait) return;
    if (e.worker.joinable()) e.worker.join();
  }
  if (e.worker.joinable()) e.worker.join();
  JitJob& j = *e.job;
  std::string err = j.err;
  bool ok = j.ok && lt_jit::load(j.code, e.has_r64, c->device, e.k, err);
  if (ok) {
    e.state = 1;
    if (j.disk_hit) c->jstats.disk_hits++;
    else c->jstats.compiles++;
  } else {
    e.state = -1;
    e.err = err;
    c->jit_err = err;
    c->jstats.failures++;
  }
  e.job.reset();  // the code object's host copy
  if (ok) jit_evict(c, key);
}

// The JIT analyze / resolve kernels of program f for a tile of Y year slots and n_rules rules
// (lt_jit.h): the instance the product would dispatch to (MAXY, RMAX buckets, series type),
// specialised on the launch's uniform values unless LT_JIT_SPEC=0 and on the scene's tables
// unless LT_JIT_SCENE=0 (or once the context holds LT_JIT_SCENE_MAX scene-specialised modules:
// a mosaic of many scenes then shares one generic module per configuration). *entry is the ready
// module, or NULL when it is still compiling (`wait` false) or failed: the tile then takes the
// precompiled kernels (launch_tile). Errors are returned only for an invalid program or HIP.
static int jit_acquire(lt_ctx* c, const lt_index* f, int Y, const lt_params* prm,
                       const lt_tile_in* in, const lt_tile_out* o, const lt::DevScene* scene,
                       bool wait, JitEntry** entry, uint64_t* key_out = nullptr) {
  *entry = nullptr;
  const int n_rules = prm->n_rules;
  const int maxy = Y <= 32 ? 32 : Y <= 48 ? 48 : 64;
  const int rmax = n_rules <= 1 ? 1 : n_rules <= 4 ? 4 : 16;
  const char* vt = lt_jit::series_type(f->out_type, n_rules);
  static const bool spec_on = !(getenv("LT_JIT_SPEC") && getenv("LT_JIT_SPEC")[0] == '0');
  static const bool scene_on = !(getenv("LT_JIT_SCENE") && getenv("LT_JIT_SCENE")[0] == '0');
  lt_jit::Spec sp;
  if (spec_on) {
    sp.on = true;
    sp.n_years = Y;
    sp.masked = in->obs_valid != nullptr || in->obs_valid_bits != nullptr;
    sp.year_out = o->val_fit || o->fit_m || o->fit_b || o->right_m || o->right_b || o->spike ||
                  o->vertex;
    sp.tl_split = tl_split_launch(c, o);
    sp.params = *prm;
    if (scene_on) sp.scene = scene;
    // the launch's output planes as constants (LT_JIT_FIELDS=0: read at run time, A/B;
    // LT_JIT_FIELDS_OR=hex: planes also treated as present, A/B of which dropped plane matters)
    static const bool fields_on = !(getenv("LT_JIT_FIELDS") && getenv("LT_JIT_FIELDS")[0] == '0');
    static const uint32_t fields_or =
        getenv("LT_JIT_FIELDS_OR") ? (uint32_t)strtoul(getenv("LT_JIT_FIELDS_OR"), nullptr, 16) : 0u;
    sp.fields_on = fields_on;
    sp.fields = fields_on ? lt_jit::spec_fields(lt_jit::out_field_mask(o) | fields_or, rmax) : 0u;
    sp.vbits = in->obs_valid_bits != nullptr && scene->n_obs <= 128;
    sp.band_pair = f->prog.n_bands == 2 &&
                   (f->prog.band_type == LT_T_I16 || f->prog.band_type == LT_T_U16) &&
                   in->band_stride == 1 && in->band_pix_stride == 2 &&
                   in->band_obs_stride % 2 == 0 && ((uintptr_t)in->obs_bands & 3) == 0;
    static const bool full_on = !(getenv("LT_JIT_FULL") && getenv("LT_JIT_FULL")[0] == '0');
    sp.full = full_on && in->n_pix % (64 * lt_jit::analyze_wpb()) == 0;
  }
  uint64_t key = lt_jit::spec_key(f->prog, maxy, rmax, vt, sp);
  auto it = c->jit.find(key);
  if (it == c->jit.end() && sp.scene) {
    int n_scene = 0;
    for (auto& kv : c->jit) n_scene += kv.second.scene_spec ? 1 : 0;
    if (n_scene >= c->jit_scene_max) {  // the generic-scene module of this configuration
      sp.scene = nullptr;
      key = lt_jit::spec_key(f->prog, maxy, rmax, vt, sp);
      it = c->jit.find(key);
    }
  }
  if (it == c->jit.end()) {
    std::string err;
    const std::string src = lt_jit::source(f->prog, maxy, rmax, vt, sp, err);
    if (src.empty()) return fail(c, LT_ERR_ARG, "%s", err.c_str());
    const int rc = device_arch(c);
    if (rc != LT_OK) return rc;
    it = c->jit.emplace(std::piecewise_construct, std::forward_as_tuple(key),
                        std::forward_as_tuple()).first;
    JitEntry& e = it->second;
    e.has_r64 = strcmp(vt, "float") == 0;
    e.scene_spec = sp.scene != nullptr;
    e.job = std::make_shared<JitJob>();
    e.job->src = src;
    e.job->arch = c->arch;
    auto run = [](std::shared_ptr<JitJob> j) {
      j->ok = lt_jit::compile(j->src, j->arch, j->code, j->disk_hit, j->err);
      j->done.store(true, std::memory_order_release);
    };
    if (wait) {
      run(e.job);
    } else {
      try {
        e.worker = std::thread(run, e.job);
      } catch (...) {  // no thread: compile here
        run(e.job);
      }
    }
  }
  JitEntry& e = it->second;
  jit_finish(c, key, e, wait);
  if (key_out) *key_out = key;
  if (e.state == 1) {
    e.last_use = ++c->jit_clock;
    *entry = &e;
  }
  return LT_OK;
}

// The fused tile `in` (obs_bands + a program) as the precompiled kernels read it, when its JIT
// kernels are not ready: a linear program as its lt_index_lin form (the precompiled fused load
// stage), any other through its index raster, written into the context's scratch of deferred-list
// set `set` by the program's load kernel on `stream` (lt_index_apply). false only on HIP errors.
static int index_apply_impl(lt_ctx* c, const lt_index* f, const lt_index_io* io, hipStream_t st);
static bool lin_tile_ok(const lt_tile_in& t, const lt_index_lin& L) {
  if (L.n_bands < 1 || L.n_bands > LT_LIN_MAX_BANDS ||
      (L.band_type != LT_T_I16 && L.band_type != LT_T_U16 && L.band_type != LT_T_U8 &&
       L.band_type != LT_T_I32) ||
      !lt_idx::is_int(L.wrap_type) || !lt_idx::ctype(L.out_type))
    return false;
  const bool planar = t.band_pix_stride == 1 && t.band_stride >= t.n_pix &&
                      t.band_obs_stride >= (int64_t)L.n_bands * t.band_stride;
  const bool interleaved = t.band_stride == 1 && t.band_pix_stride == L.n_bands &&
                           t.band_obs_stride >= (int64_t)L.n_bands * t.n_pix;
  if (!planar && !interleaved) return false;
  const int64_t esz = (int64_t)lt_idx::type_size(L.band_type);
  if (interleaved && L.n_bands == 2 && esz == 2 &&
      ((uintptr_t)t.obs_bands % 4 != 0 || t.band_obs_stride % 2 != 0))
    return false;
  return true;
}
static int jit_fallback_tile(lt_ctx* c, const lt_tile_in* in, int n_obs, int set,
                             hipStream_t stream, lt_tile_in& alt) {
  alt = *in;
  alt.index = nullptr;
  const lt_index* f = in->index;
  lt_index_lin lin;
  if (lt_idx::linearize(f->prog, lin) && lin_tile_ok(alt, lin)) {
    alt.lin = lin;
    return LT_OK;
  }
  const size_t need = (size_t)n_obs * (size_t)in->stride * lt_idx::type_size(f->out_type);
  if (c->iscratch_bytes[set] < need) {
    if (c->d_iscratch[set]) {
      HIP_OR_FAIL(c, hipStreamSynchronize(stream));
      HIP_OR_FAIL(c, hipFree(c->d_iscratch[set]));
    }
    c->d_iscratch[set] = nullptr;
    c->iscratch_bytes[set] = 0;
    HIP_OR_FAIL(c, hipMalloc(&c->d_iscratch[set], need));
    c->iscratch_bytes[set] = need;
  }
  lt_index_io io;
  io.n_pix = in->n_pix;
  io.n_obs = n_obs;
  io.obs_stride = in->band_obs_stride;
  io.band_stride = in->band_stride;
  io.band_pix_stride = in->band_pix_stride;
  io.out_stride = in->stride;  // the index raster shares the mask planes' row stride
  io.bands = in->obs_bands;
  io.out = c->d_iscratch[set];
  if (n_obs > 0) {
    const int rc = index_apply_impl(c, f, &io, stream);
    if (rc != LT_OK) return rc;
  }
  alt.obs_bands = nullptr;
  alt.obs_index = c->d_iscratch[set];
  alt.index_type = f->out_type;
  return LT_OK;
}

// set `set`'s compact trendline buffers for defer_cap pixels and Y year slots (Y-1 segments),
// and the expand stream; a buffer still read by an earlier tile's expand kernel is freed only
// after it (the set's last user is ordered before this tile by ev_resolved, but a resize frees)
static int tl_buffers(lt_ctx* c, int set, int Y) {
  if (!c->xstream) {
    int least = 0, greatest = 0;
    HIP_OR_FAIL(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
    const char* pr = getenv("LT_EXPAND_PRIORITY");  // high / normal / low (A/B runs)
    const int prio = pr && strcmp(pr, "high") == 0 ? greatest
                     : pr && strcmp(pr, "low") == 0 ? least : 0;
    HIP_OR_FAIL(c, hipStreamCreateWithPriority(&c->xstream, hipStreamNonBlocking, prio));
    HIP_OR_FAIL(c, hipEventCreateWithFlags(&c->ev_xdone, hipEventDisableTiming));
    for (int s = 0; s < lt_ctx::kSets; s++)
      HIP_OR_FAIL(c, hipEventCreateWithFlags(&c->ev_rdone[s], hipEventDisableTiming));
  }
  const int segs = Y > 1 ? Y - 1 : 1;
  if (c->tl_cap[set] >= c->defer_cap && c->tl_segs[set] >= segs) return LT_OK;
  HIP_OR_FAIL(c, hipStreamSynchronize(c->xstream));
  if (c->d_tl_bits[set]) HIP_OR_FAIL(c, hipFree(c->d_tl_bits[set]));
  if (c->d_tl_eqn[set]) HIP_OR_FAIL(c, hipFree(c->d_tl_eqn[set]));
  c->d_tl_bits[set] = nullptr;
  c->d_tl_eqn[set] = nullptr;
  c->tl_cap[set] = 0;
  HIP_OR_FAIL(c, hipMalloc((void**)&c->d_tl_bits[set], 4 * sizeof(uint64_t) * (size_t)c->defer_cap));
  HIP_OR_FAIL(c, hipMalloc((void**)&c->d_tl_eqn[set],
                           2 * sizeof(double) * (size_t)segs * (size_t)c->defer_cap));
  c->tl_cap[set] = c->defer_cap;
  c->tl_segs[set] = segs;
  return LT_OK;
}

// One tile's stages: the analyze kernel on `stream`, the resolve kernels (its deferred pixels) on
// `rstream` once the analyze kernel is done; deferred-pixel list / counters set `set`.
static int launch_tile(lt_ctx* c, const lt_params* prm, const lt_tile_in* in,
                       const lt_tile_out* out, int Y, hipStream_t stream, hipStream_t rstream,
                       int set) {
  int64_t* dl = c->d_defer + (size_t)set * 2 * c->defer_cap;
  // per-year planes requested: with the compact trendline (default) the analyze / resolve
  // stages leave per-pixel words and segment eqns and trendline_expand_kernel writes every plane
  // (spike / vertex included); else the year-major loop writes the planes and the spike / vertex
  // planes go through per-pixel year flags ([2][n_pix] of this set)
  const bool tl = tl_split_launch(c, out);
  uint64_t* yf = (!tl && (out->spike || out->vertex))
                     ? c->d_yflags + (size_t)set * 2 * c->defer_cap : nullptr;
  if (tl) {
    const int rc = tl_buffers(c, set, Y);
    if (rc != LT_OK) return rc;
  }
  unsigned long long* dn = c->d_ndefer + 4 * set;
  // [0]/[2]: deferred-pixel counts of the binary32 / binary64 lists (stage 1), [1]/[3]: the
  // resolve launches' work counters
  HIP_OR_FAIL(c, hipMemsetAsync(dn, 0, 4 * sizeof(unsigned long long), stream));
  EventPair* ep[3] = {nullptr, nullptr, nullptr};
  if (c->timing) {
    while (c->pool.size() < c->used + 3) {  // grow first: pointers into the pool stay valid
      EventPair np;
      HIP_OR_FAIL(c, hipEventCreate(&np.start));
      HIP_OR_FAIL(c, hipEventCreate(&np.stop));
      c->pool.push_back(np);
    }
    ep[0] = &c->pool[c->used++];
    ep[1] = &c->pool[c->used++];
    ep[2] = &c->pool[c->used++];
  }
  if (ep[0]) HIP_OR_FAIL(c, hipEventRecord(ep[0]->start, stream));
  const int64_t nwave = (in->n_pix + 63) / 64;
  if (nwave > 0x7fffffff) return fail(c, LT_ERR_LIMIT, "tile too large%s");
  lt::TileLaunch l{c->d_scene, prm, in, out, c->d_xtab, dl, dn, yf, Y, c->device, stream};
  if (tl) {
    l.tl_bits = c->d_tl_bits[set];
    l.tl_eqn = c->d_tl_eqn[set];
  }
  const lt_jit_kernels* jk = nullptr;
  JitEntry* je = nullptr;
  lt_tile_in alt;  // the tile as the precompiled kernels read it (JIT kernels not ready)
  if (in->obs_bands && in->index) {  // a program inlined into JIT kernels (lt_jit.h)
    const int rc = jit_acquire(c, in->index, Y, prm, in, out, c->h_scene,
                               c->jit_mode == LT_JIT_SYNC, &je);
    if (rc != LT_OK) return rc;
    if (je) {
      jk = &je->k;
      c->jstats.jit_tiles++;
    } else {  // still compiling or failed: the precompiled kernels, same results
      const int rf = jit_fallback_tile(c, in, c->h_scene->n_obs, set, stream, alt);
      if (rf != LT_OK) return rf;
      l.in = &alt;
      c->jstats.fallback_tiles++;
    }
  }
  // the JIT kernels' one argument, as the product kernels get it (lt_kernels.h kernel_args)
  auto jit_launch = [&](hipFunction_t f, unsigned grid, int64_t* list,
                        unsigned long long* counters, hipStream_t s, int wpb = 1) -> hipError_t {
    lt::KernelArgs a{c->d_scene, *prm, *in, *out, c->d_xtab, list, counters, yf, l.tl_bits,
                     l.tl_eqn};
    size_t sz = sizeof a;
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                   HIP_LAUNCH_PARAM_END};
    return hipModuleLaunchKernel(f, grid, 1, 1, 64 * wpb, 1, 1, 0, s, nullptr, cfg);
  };
  // LT_SYNC_LAUNCH=1 (debugging): wait for each stage and report a fault against it
  static const bool sync_each = getenv("LT_SYNC_LAUNCH") && getenv("LT_SYNC_LAUNCH")[0] == '1';
  if (jk)
    HIP_OR_FAIL(c, jit_launch(jk->analyze, (unsigned)((nwave + jk->wpb - 1) / jk->wpb), dl, dn,
                              stream, jk->wpb));
  else
    HIP_OR_FAIL(c, lt::launch_analyze(l));
  if (sync_each) HIP_OR_FAIL(c, hipStreamSynchronize(stream));
  if (ep[0]) HIP_OR_FAIL(c, hipEventRecord(ep[0]->stop, stream));
  if (rstream != stream) {
    HIP_OR_FAIL(c, hipEventRecord(c->ev_analyzed[set], stream));
    HIP_OR_FAIL(c, hipStreamWaitEvent(rstream, c->ev_analyzed[set], 0));
  }
  if (ep[1]) HIP_OR_FAIL(c, hipEventRecord(ep[1]->start, rstream));
  stream = rstream;  // the resolve launches below
  l.stream = rstream;
  if (jk) {  // the deferred lists, as launch_resolve_instance launches them
    const unsigned g0 = jk->resolve_grid < (unsigned)nwave ? jk->resolve_grid : (unsigned)nwave;
    HIP_OR_FAIL(c, jit_launch(jk->resolve, g0, dl, dn, stream));
    // the second list (values binary32 cannot hold): empty for an int16 series (not launched,
    // as launch_resolve_instance does), the binary64 resolve for a binary32 one, the same
    // kernel for a binary64 one
    const bool i16 = in->index->out_type == LT_T_I16;
    if (!i16) {
      hipFunction_t f64 = jk->resolve64 ? jk->resolve64 : jk->resolve;
      const unsigned gw = jk->resolve64 ? jk->resolve64_grid : jk->resolve_grid;
      const unsigned g1 = gw < (unsigned)nwave ? gw : (unsigned)nwave;
      HIP_OR_FAIL(c, jit_launch(f64, g1, dl + in->n_pix, dn + 2, stream));
    }
  } else {
    HIP_OR_FAIL(c, lt::launch_resolve(l));
  }
  if (sync_each) HIP_OR_FAIL(c, hipStreamSynchronize(stream));
  if (tl) {  // every pixel's compact trendline is in (analyze + resolve): the year rows
    if (ep[1]) HIP_OR_FAIL(c, hipEventRecord(ep[1]->stop, rstream));
    HIP_OR_FAIL(c, hipEventRecord(c->ev_rdone[set], rstream));
    HIP_OR_FAIL(c, hipStreamWaitEvent(c->xstream, c->ev_rdone[set], 0));
    if (ep[2]) HIP_OR_FAIL(c, hipEventRecord(ep[2]->start, c->xstream));
    if (Y > 0) {
      const int64_t nb = (in->n_pix + kBlock - 1) / kBlock * ((Y + kYC - 1) / kYC);
      if (nb > 0x7fffffff) return fail(c, LT_ERR_LIMIT, "tile too large for the expand grid%s");
      hipLaunchKernelGGL(trendline_expand_kernel, dim3((unsigned)nb), dim3(kBlock), 0,
                         c->xstream, c->d_scene, l.tl_bits, l.tl_eqn, in->n_pix, Y, *out);
    }
    HIP_OR_FAIL(c, hipGetLastError());
    if (ep[2]) HIP_OR_FAIL(c, hipEventRecord(ep[2]->stop, c->xstream));
    // the set (and the expand kernel's reads of it) is free again after this point
    HIP_OR_FAIL(c, hipEventRecord(c->ev_resolved[set], c->xstream));
    HIP_OR_FAIL(c, hipEventRecord(c->ev_xdone, c->xstream));
    c->x_used = true;
    c->last_stage = c->xstream;
    if (je) {  // the module may be unloaded (jit_evict) only after this launch
      if (!je->ev_last)
        HIP_OR_FAIL(c, hipEventCreateWithFlags(&je->ev_last, hipEventDisableTiming));
      HIP_OR_FAIL(c, hipEventRecord(je->ev_last, rstream));
    }
    c->last_set = set;
    c->launches++;
    return LT_OK;
  }
  if (yf) {  // every pixel's flags are in (analyze + resolve): expand them into the planes
    const bool v4 = ((uintptr_t)out->spike % 4 == 0) && ((uintptr_t)out->vertex % 4 == 0) &&
                    out->stride % 4 == 0;
    const int64_t nthr = v4 ? (in->n_pix + 3) / 4 : in->n_pix;
    dim3 eg((unsigned)((nthr + kBlock - 1) / kBlock)), eb(kBlock);
    if (v4)
      hipLaunchKernelGGL((year_flags_kernel<true>), eg, eb, 0, stream, yf, in->n_pix, Y,
                         out->spike, out->vertex, out->stride);
    else
      hipLaunchKernelGGL((year_flags_kernel<false>), eg, eb, 0, stream, yf, in->n_pix, Y,
                         out->spike, out->vertex, out->stride);
  }
  HIP_OR_FAIL(c, hipGetLastError());
  if (ep[1]) HIP_OR_FAIL(c, hipEventRecord(ep[1]->stop, rstream));
  if (ep[2]) {  // no expand stage: an empty interval
    HIP_OR_FAIL(c, hipEventRecord(ep[2]->start, rstream));
    HIP_OR_FAIL(c, hipEventRecord(ep[2]->stop, rstream));
  }
  HIP_OR_FAIL(c, hipEventRecord(c->ev_resolved[set], rstream));
  c->last_stage = rstream;
  if (je) {  // the module may be unloaded (jit_evict) only after this launch
    if (!je->ev_last)
      HIP_OR_FAIL(c, hipEventCreateWithFlags(&je->ev_last, hipEventDisableTiming));
    HIP_OR_FAIL(c, hipEventRecord(je->ev_last, rstream));
  }
  c->last_set = set;
  c->launches++;
  return LT_OK;
}

// The scene's device table (lt_pixel.h DevScene), validated: scene metadata of lt_scene, the
// rule count of prm, and the winner of every year when no observation is masked (pick_winners'
// first observation, input order, at minimal |days|, as the kernels pick it)
static int scene_from(lt_ctx* c, const lt_scene* sc, const lt_params* prm, lt::DevScene& tmp) {
  const int K = sc->n_obs, Y = sc->n_years;
  if (K < 0 || K > LT_MAX_OBS || Y < 0 || Y > LT_MAX_YEARS)
    return fail(c, LT_ERR_LIMIT, "scene exceeds LT_MAX_OBS/LT_MAX_YEARS%s");
  if (prm->n_rules < 0 || prm->n_rules > LT_MAX_RULES)
    return fail(c, LT_ERR_LIMIT, "too many rules%s");
  if (Y > 0 && (!sc->year || !sc->slot_begin || !sc->order || !sc->dist))
    return fail(c, LT_ERR_ARG, "scene arrays missing%s");
  if (Y > 0 && (sc->slot_begin[0] != 0 || sc->slot_begin[Y] != K))
    return fail(c, LT_ERR_ARG, "slot_begin must span [0, n_obs]%s");
  for (int y = 0; y < Y; y++) {
    if (sc->slot_begin[y + 1] < sc->slot_begin[y])
      return fail(c, LT_ERR_ARG, "slot_begin not monotone%s");
    if (y > 0 && sc->year[y] <= sc->year[y - 1])
      return fail(c, LT_ERR_ARG, "years must be strictly ascending%s");
  }
  for (int k = 0; k < K; k++) {
    if (sc->order[k] < 0 || sc->order[k] >= K)
      return fail(c, LT_ERR_ARG, "order[] out of range%s");
    if (sc->dist[k] < 0) return fail(c, LT_ERR_ARG, "negative dist%s");
  }
  if (Y > 0 && sc->year[Y - 1] - sc->year[0] > 255)
    return fail(c, LT_ERR_LIMIT, "year span above 255%s");
  memset(&tmp, 0, sizeof tmp);
  tmp.n_obs = K;
  tmp.n_years = Y;
  for (int y = 0; y < Y; y++) {
    tmp.year[y] = sc->year[y];
    if (sc->feb29_bad && sc->feb29_bad[y]) tmp.feb29_mask |= 1ull << y;
  }
  for (int y = 0; y <= Y; y++) tmp.slot_begin[y] = Y > 0 ? sc->slot_begin[y] : 0;
  for (int k = 0; k < K; k++) {
    tmp.order[k] = sc->order[k];
    tmp.dist[k] = sc->dist[k];
  }
  for (int y = 0; y < Y; y++) {  // first obs (input order) at minimal |days|, as the kernels pick
    int best = -1, bd = 0x7fffffff;
    for (int k = tmp.slot_begin[y]; k < tmp.slot_begin[y + 1]; k++)
      if (tmp.dist[k] < bd) {
        bd = tmp.dist[k];
        best = tmp.order[k];
      }
    tmp.winner_all[y] = best;
  }
  return LT_OK;
}

int lt_analyze_tiles(lt_ctx* c, const lt_scene* sc, const lt_params* prm, int n_tiles,
                     const lt_tile_in* ins, const lt_tile_out* outs, void* stream_) {
  return lt_analyze_tiles_after(c, sc, prm, n_tiles, ins, outs, nullptr, stream_);
}

int lt_analyze_tiles_after(lt_ctx* c, const lt_scene* sc, const lt_params* prm, int n_tiles,
                           const lt_tile_in* ins, const lt_tile_out* outs, void* const* ready,
                           void* stream_) {
  return lt_analyze_tiles_ev(c, sc, prm, n_tiles, ins, outs, ready, nullptr, 1, stream_);
}

int lt_analyze_tiles_ev(lt_ctx* c, const lt_scene* sc, const lt_params* prm, int n_tiles,
                        const lt_tile_in* ins, const lt_tile_out* outs, void* const* ready,
                        void* const* done, int32_t join, void* stream_) {
  if (!c) return LT_ERR_ARG;
  if (!sc || !prm || n_tiles < 0 || (n_tiles > 0 && (!ins || !outs)))
    return fail(c, LT_ERR_ARG, "null argument%s");
  int64_t cap = 0;
  for (int t = 0; t < n_tiles; t++) {
    const int rc = check_tile(c, &ins[t], &outs[t]);
    if (rc != LT_OK) return rc;
    cap = ins[t].n_pix > cap ? ins[t].n_pix : cap;
  }
  if (cap == 0) return LT_OK;
  lt::DevScene tmp;
  {
    const int rc = scene_from(c, sc, prm, tmp);
    if (rc != LT_OK) return rc;
  }
  const int Y = tmp.n_years;
  HIP_OR_FAIL(c, hipSetDevice(c->device));
  hipStream_t stream = (hipStream_t)stream_;

  // scene upload (skipped when identical to the resident one)
  if (!c->scene_valid || memcmp(&tmp, c->h_scene, sizeof tmp) != 0) {
    // an earlier call, possibly on another stream, may still be reading d_scene: its last tile's
    // resolve (side stream, in order, after every analyze it waited for) marks the end of all of
    // that work, so the copy waits for it
    bool any = false;
    for (int s = 0; s < lt_ctx::kSets; s++) any = any || c->set_used[s];
    if (any) HIP_OR_FAIL(c, hipStreamWaitEvent(stream, c->ev_resolved[c->last_set], 0));
    HIP_OR_FAIL(c, hipEventSynchronize(c->scene_copied));  // staging buffer free again
    memcpy(c->h_scene, &tmp, sizeof tmp);
    HIP_OR_FAIL(c, hipMemcpyAsync(c->d_scene, c->h_scene, sizeof tmp, hipMemcpyHostToDevice,
                                  stream));
    HIP_OR_FAIL(c, hipEventRecord(c->scene_copied, stream));
    c->scene_valid = true;
  }

  // deferred-pixel lists: kSets sets (round robin over tiles), sized for the largest tile seen
  if (c->defer_cap < cap) {
    // a smaller list may still be read by an earlier call's resolve on the side stream
    if (c->side) HIP_OR_FAIL(c, hipStreamSynchronize(c->side));
    if (c->d_defer) HIP_OR_FAIL(c, hipFree(c->d_defer));
    c->d_defer = nullptr;
    if (c->d_yflags) HIP_OR_FAIL(c, hipFree(c->d_yflags));
    c->d_yflags = nullptr;
    const size_t ns = lt_ctx::kSets;
    HIP_OR_FAIL(c, hipMalloc((void**)&c->d_defer, ns * 2 * sizeof(int64_t) * (size_t)cap));
    HIP_OR_FAIL(c, hipMalloc((void**)&c->d_yflags, ns * 2 * sizeof(uint64_t) * (size_t)cap));
    if (!c->d_ndefer)
      HIP_OR_FAIL(c, hipMalloc((void**)&c->d_ndefer, ns * 4 * sizeof(unsigned long long)));
    c->defer_cap = cap;
  }
  if (!c->side) {
    // the resolve stage's stream has the lowest priority: its few long, latency-bound waves then
    // take CU slots only when the next tile's analyze waves leave them (the drain of a launch),
    // instead of displacing them at the launch's start (kernel trace r04_run1: a resolve launch
    // that got its slots first cost the analyze launch beside it 0.25-0.29 ms; one that did not
    // ran in its shadow for free). LT_RESOLVE_PRIORITY=normal keeps the default (A/B runs).
    int least = 0, greatest = 0;
    HIP_OR_FAIL(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
    const char* pr = getenv("LT_RESOLVE_PRIORITY");
    const bool normal = pr && strcmp(pr, "normal") == 0;
    HIP_OR_FAIL(c, hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, normal ? 0 : least));
    for (int s = 0; s < lt_ctx::kSets; s++) {
      HIP_OR_FAIL(c, hipEventCreateWithFlags(&c->ev_analyzed[s], hipEventDisableTiming));
      HIP_OR_FAIL(c, hipEventCreateWithFlags(&c->ev_resolved[s], hipEventDisableTiming));
    }
    const char* ns = getenv("LT_DEFER_SETS");
    if (ns && atoi(ns) >= 2 && atoi(ns) <= lt_ctx::kSets) c->n_sets = atoi(ns);
  }
  // Tile t: analyze on `stream`, resolve on the context's side stream, so tile t's resolve runs
  // beside tile t+1's analyze (the resolve is a few long waves: latency, not throughput). A set
  // is reused n_sets tiles later, after its tile's resolve: with two sets tile t+2's analyze
  // waited for tile t's resolve, whose waves get CU slots only in tile t+1's drain (kernel trace
  // r04_run1: 0.37 ms of a 22 ms step with the GPU nearly idle). At the end `stream` waits for
  // the last resolve, so every output is complete in `stream` order when the call's work is done.
  for (int t = 0; t < n_tiles; t++) {
    if (ins[t].n_pix == 0) continue;
    const int set = c->next_set;
    c->next_set = (set + 1) % c->n_sets;
    if (c->set_used[set]) HIP_OR_FAIL(c, hipStreamWaitEvent(stream, c->ev_resolved[set], 0));
    if (ready && ready[t]) HIP_OR_FAIL(c, hipStreamWaitEvent(stream, (hipEvent_t)ready[t], 0));
    const int rc = launch_tile(c, prm, &ins[t], &outs[t], Y, stream, c->side, set);
    if (rc != LT_OK) return rc;
    c->set_used[set] = true;
    // the caller's per-tile event: after the tile's last stage (ev_resolved was just recorded on
    // that stage's stream), e.g. for a label exchange that waits for this tile alone
    if (done && done[t]) HIP_OR_FAIL(c, hipEventRecord((hipEvent_t)done[t], c->last_stage));
  }
  if (!join) return LT_OK;
  // (the last tile's launch recorded ev_resolved after its last stage: the resolve kernels, or
  // the trendline expand kernel on the expand stream)
  HIP_OR_FAIL(c, hipStreamWaitEvent(stream, c->ev_resolved[c->last_set], 0));
  return LT_OK;
}

int lt_analyze_tile(lt_ctx* c, const lt_scene* sc, const lt_params* prm, const lt_tile_in* in,
                    const lt_tile_out* out, void* stream_) {
  if (!c) return LT_ERR_ARG;
  if (!in || !out) return fail(c, LT_ERR_ARG, "null argument%s");
  return lt_analyze_tiles(c, sc, prm, 1, in, out, stream_);
}

int lt_ctx_last_deferred(lt_ctx* c, int64_t* n_deferred) {
  if (!c || !n_deferred) return LT_ERR_ARG;
  *n_deferred = 0;
  if (!c->d_ndefer) return LT_OK;
  HIP_OR_FAIL(c, hipSetDevice(c->device));
  unsigned long long v[4] = {0, 0, 0, 0};
  HIP_OR_FAIL(c, hipDeviceSynchronize());  // the counters of the last tile's set
  HIP_OR_FAIL(c, hipMemcpy(v, c->d_ndefer + 4 * c->last_set, sizeof v, hipMemcpyDeviceToHost));
  *n_deferred = (int64_t)(v[0] + v[2]);
  return LT_OK;
}

int lt_raster_assemble(lt_ctx* c, const lt_raster_job* jobs, int n_jobs, void* stream_) {
  if (!c) return LT_ERR_ARG;
  if (n_jobs < 0 || (n_jobs > 0 && !jobs)) return fail(c, LT_ERR_ARG, "null argument%s");
  for (int k = 0; k < n_jobs; k++) {
    const lt_raster_job& J = jobs[k];
    if (J.n_pix < 0 || J.n_out < 0 || (!J.out && J.n_out > 0))
      return fail(c, LT_ERR_ARG, "bad raster job sizes%s");
    if (!J.dest && J.n_out != J.n_pix)
      return fail(c, LT_ERR_ARG, "identity offsets need n_out == n_pix%s");
    if (J.sel_kind < LT_SEL_ALL || J.sel_kind > LT_SEL_EQUALS || (J.sel_kind != LT_SEL_ALL && !J.sel))
      return fail(c, LT_ERR_ARG, "bad selector%s");
    if (J.plane && J.plane_type != LT_T_I32 && J.plane_type != LT_T_F64 &&
        J.plane_type != LT_T_U8 && J.plane_type != LT_T_I16)
      return fail(c, LT_ERR_ARG, "bad plane type%s");
    if (J.mode == LT_RASTER_REFERENCE ? (J.out_type != LT_T_U8 || !lt_idx::ctype(J.holder_type))
                                      : (J.mode != LT_RASTER_TYPED ||
                                         (J.out_type != LT_T_I32 && J.out_type != LT_T_F64 &&
                                          J.out_type != LT_T_U8)))
      return fail(c, LT_ERR_ARG, "bad raster mode / type%s");
  }
  HIP_OR_FAIL(c, hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream_;
  for (int k = 0; k < n_jobs; k++) {
    const lt_raster_job& J = jobs[k];
    auto grid = [](int64_t n) {
      const int64_t b = (n + kBlock - 1) / kBlock;
      return dim3((unsigned)(b < 65536 ? (b > 0 ? b : 1) : 65536));
    };
    if (J.dest) {
      if (J.n_out > 0)
        hipLaunchKernelGGL(raster_fill_kernel, grid(J.n_out), dim3(kBlock), 0, st, J);
      if (J.n_pix > 0)
        hipLaunchKernelGGL(raster_scatter_kernel, grid(J.n_pix), dim3(kBlock), 0, st, J, false);
    } else if (J.n_pix > 0) {
      hipLaunchKernelGGL(raster_scatter_kernel, grid(J.n_pix), dim3(kBlock), 0, st, J, true);
    }
    HIP_OR_FAIL(c, hipGetLastError());
  }
  return LT_OK;
}

int lt_winner_presence(lt_ctx* c, const int16_t* winner, int64_t stride, int32_t n_years,
                       int64_t n_pix, int32_t n_obs, uint32_t* bits, void* stream_) {
  if (!c) return LT_ERR_ARG;
  if (n_years < 0 || n_years > LT_MAX_YEARS || n_obs < 0 || n_obs > LT_MAX_OBS || n_pix < 0 ||
      stride < n_pix)
    return fail(c, LT_ERR_ARG, "bad presence sizes%s");
  if (n_obs == 0) return LT_OK;
  if (!bits || (n_years > 0 && n_pix > 0 && !winner)) return fail(c, LT_ERR_ARG, "null argument%s");
  HIP_OR_FAIL(c, hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream_;
  HIP_OR_FAIL(c, hipMemsetAsync(bits, 0, sizeof(uint32_t) * ((n_obs + 31) / 32), st));
  if (n_years == 0 || n_pix == 0) return LT_OK;
  const int64_t b = (n_pix + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(winner_presence_kernel, dim3((unsigned)(b < 4096 ? b : 4096)), dim3(kBlock), 0,
                     st, winner, stride, (int)n_years, n_pix, (int)n_obs, bits);
  HIP_OR_FAIL(c, hipGetLastError());
  return LT_OK;
}

int lt_label_tile(lt_ctx* c, const lt_label_in* in, const lt_params* prm, const lt_tile_out* out,
                  void* stream_) {
  if (!c) return LT_ERR_ARG;
  if (!in || !prm || !out) return fail(c, LT_ERR_ARG, "null argument%s");
  if (in->n_pix < 0 || in->stride < in->n_pix || out->stride < in->n_pix)
    return fail(c, LT_ERR_ARG, "bad n_pix/stride%s");
  if (in->n_years < 0 || in->n_years > LT_MAX_YEARS || prm->n_rules < 0 ||
      prm->n_rules > LT_MAX_RULES)
    return fail(c, LT_ERR_LIMIT, "too many years or rules%s");
  if (in->n_pix == 0) return LT_OK;
  if (in->n_years > 0 && (!in->year || !in->val_fit || !in->vertex))
    return fail(c, LT_ERR_ARG, "year/val_fit/vertex required%s");
  HIP_OR_FAIL(c, hipSetDevice(c->device));
  YearArg ya;
  memset(&ya, 0, sizeof ya);
  for (int y = 0; y < in->n_years; y++) ya.year[y] = in->year[y];
  const int64_t nblk = (in->n_pix + kBlock - 1) / kBlock;
  if (nblk > 0x7fffffff) return fail(c, LT_ERR_LIMIT, "tile too large%s");
  hipLaunchKernelGGL(label_kernel, dim3((unsigned)nblk), dim3(kBlock), 0, (hipStream_t)stream_,
                     ya, in->n_years, *prm, *in, *out);
  HIP_OR_FAIL(c, hipGetLastError());
  return LT_OK;
}

int lt_ctx_set_jit_mode(lt_ctx* c, int32_t mode) {
  if (!c) return LT_ERR_ARG;
  if (mode != LT_JIT_SYNC && mode != LT_JIT_ASYNC) return fail(c, LT_ERR_ARG, "bad JIT mode%s");
  c->jit_mode = mode;
  return LT_OK;
}

int lt_jit_prepare(lt_ctx* c, const lt_scene* sc, const lt_params* prm, const lt_tile_in* in,
                   const lt_tile_out* out, int32_t wait) {
  if (!c) return LT_ERR_ARG;
  if (!sc || !prm || !in || !out) return fail(c, LT_ERR_ARG, "null argument%s");
  if (!(in->obs_bands && in->index)) return LT_OK;  // no program: no JIT kernels
  lt::DevScene tmp;
  int rc = scene_from(c, sc, prm, tmp);
  if (rc != LT_OK) return rc;
  HIP_OR_FAIL(c, hipSetDevice(c->device));
  JitEntry* e = nullptr;
  uint64_t key = 0;
  rc = jit_acquire(c, in->index, tmp.n_years, prm, in, out, &tmp, wait != 0, &e, &key);
  if (rc != LT_OK) return rc;
  auto it = c->jit.find(key);
  if (it != c->jit.end() && it->second.state < 0)
    return fail(c, LT_ERR_JIT, "%s", it->second.err.c_str());
  return LT_OK;
}

int lt_ctx_jit_stats(lt_ctx* c, lt_jit_stats* out, char* last_error, int64_t cap) {
  if (!c || !out) return LT_ERR_ARG;
  // finish compiles that are done (the module is loaded on this thread)
  for (auto& kv : c->jit)
    if (kv.second.state == 0) jit_finish(c, kv.first, kv.second, false);
  *out = c->jstats;
  out->modules = 0;
  out->pending = 0;
  for (auto& kv : c->jit) {
    out->modules += kv.second.state == 1 ? 1 : 0;
    out->pending += kv.second.state == 0 ? 1 : 0;
  }
  if (last_error && cap > 0) {
    const size_t n = c->jit_err.size() < (size_t)(cap - 1) ? c->jit_err.size() : (size_t)(cap - 1);
    memcpy(last_error, c->jit_err.data(), n);
    last_error[n] = 0;
  }
  return LT_OK;
}

int lt_jit_source(const lt_scene* sc, const lt_params* prm, const lt_index_prog* prog,
                  int32_t masked, int32_t year_out, int32_t flags, char* buf, int64_t cap) {
  if (!sc || !prm || !prog) return LT_ERR_ARG;
  lt::DevScene tmp;
  if (scene_from(nullptr, sc, prm, tmp) != LT_OK) return LT_ERR_ARG;
  const int Y = tmp.n_years, n_rules = prm->n_rules;
  const int maxy = Y <= 32 ? 32 : Y <= 48 ? 48 : 64;
  const int rmax = n_rules <= 1 ? 1 : n_rules <= 4 ? 4 : 16;
  lt_jit::Spec sp;
  if (flags & LT_JIT_SRC_SPEC) {
    sp.on = true;
    sp.n_years = Y;
    sp.masked = masked != 0;
    sp.year_out = year_out != 0;
    sp.tl_split = sp.year_out && getenv("LT_TL_SPLIT") && getenv("LT_TL_SPLIT")[0] == '1';
    sp.params = *prm;
    if (flags & LT_JIT_SRC_SCENE) sp.scene = &tmp;
    if (flags & LT_JIT_SRC_FIELDS) {  // the output-field mask in bits 8.. of flags
      sp.fields_on = true;
      sp.fields = lt_jit::spec_fields((uint32_t)flags >> 8, rmax);
      sp.vbits = masked != 0 && tmp.n_obs <= 128;  // the bit planes bench.py and the job pass
      // bench.py's pixel-interleaved int16 pair
      sp.band_pair = prog->n_bands == 2 &&
                     (prog->band_type == LT_T_I16 || prog->band_type == LT_T_U16);
      sp.full = true;  // bench.py's tiles are whole waves
    }
  }
  std::string err;
  const char* vt = lt_jit::series_type(prog->out_type, n_rules);
  const std::string src = lt_jit::source(*prog, maxy, rmax, vt, sp, err);
  if (src.empty()) return LT_ERR_ARG;
  // the context's module key of this specialisation (hashed here too, so the host-only tests
  // exercise it)
  volatile uint64_t key = lt_jit::spec_key(*prog, maxy, rmax, vt, sp);
  (void)key;
  if (buf && cap > 0) {
    const size_t n = src.size() < (size_t)(cap - 1) ? src.size() : (size_t)(cap - 1);
    memcpy(buf, src.data(), n);
    buf[n] = 0;
  }
  return (int)src.size();
}

}  // extern "C"

// ---- load stage (lt_index.h) ------------------------------------------------------------------
int lt_index_codegen(const lt_index_prog* prog, char* buf, int64_t cap) {
  if (!prog) return LT_ERR_ARG;
  std::string err;
  const std::string src = lt_idx::codegen(*prog, err);
  if (src.empty()) return LT_ERR_ARG;
  if (buf && cap > 0) {
    const size_t n = src.size() < (size_t)(cap - 1) ? src.size() : (size_t)(cap - 1);
    memcpy(buf, src.data(), n);
    buf[n] = 0;
  }
  return (int)src.size();
}

int lt_index_compile(lt_ctx* c, const lt_index_prog* prog, lt_index** out) {
  if (!c) return LT_ERR_ARG;
  if (!prog || !out) return fail(c, LT_ERR_ARG, "null argument%s");
  *out = nullptr;
  std::string err;
  const std::string src = lt_idx::codegen(*prog, err);
  if (src.empty()) return fail(c, LT_ERR_ARG, "%s", err.c_str());
  auto it = c->index_fns.find(src);
  if (it != c->index_fns.end()) {
    *out = it->second;
    return LT_OK;
  }
  HIP_OR_FAIL(c, hipSetDevice(c->device));
  hipDeviceProp_t prop;
  HIP_OR_FAIL(c, hipGetDeviceProperties(&prop, c->device));
  const std::string arch = std::string("--offload-arch=") + prop.gcnArchName;
  hiprtcProgram rp;
  if (hiprtcCreateProgram(&rp, src.c_str(), "lt_index.hip", 0, nullptr, nullptr) !=
      HIPRTC_SUCCESS)
    return fail(c, LT_ERR_JIT, "hiprtcCreateProgram failed%s");
  const char* opts[] = {arch.c_str(), "-O3", "-ffp-contract=off"};
  const hiprtcResult rc = hiprtcCompileProgram(rp, 3, opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(rp, &n);
    std::string log(n, '\0');
    if (n) hiprtcGetProgramLog(rp, &log[0]);
    hiprtcDestroyProgram(&rp);
    return fail(c, LT_ERR_JIT, "hiprtc: %s", log.c_str());
  }
  size_t code_size = 0;
  hiprtcGetCodeSize(rp, &code_size);
  std::vector<char> code(code_size);
  hiprtcGetCode(rp, code.data());
  hiprtcDestroyProgram(&rp);
  lt_index* f = new lt_index();
  f->n_bands = prog->n_bands;
  f->band_type = prog->band_type;
  f->out_type = prog->out_type;
  f->prog = *prog;
  if (hipModuleLoadData(&f->mod, code.data()) != hipSuccess ||
      hipModuleGetFunction(&f->fn, f->mod, "lt_index_kernel") != hipSuccess ||
      hipModuleGetFunction(&f->fn4, f->mod, "lt_index_kernel4") != hipSuccess ||
      hipModuleGetFunction(&f->fn4i, f->mod, "lt_index_kernel4i") != hipSuccess) {
    if (f->mod) (void)hipModuleUnload(f->mod);
    delete f;
    return fail(c, LT_ERR_JIT, "module load failed%s");
  }
  c->index_fns[src] = f;
  *out = f;
  return LT_OK;
}

int lt_index_linearize(const lt_index_prog* prog, lt_index_lin* out) {
  if (!prog || !out) return LT_ERR_ARG;
  return lt_idx::linearize(*prog, *out) ? LT_OK : LT_ERR_ARG;
}

int lt_index_apply(lt_ctx* c, const lt_index* f, const lt_index_io* io, void* stream_) {
  if (!c) return LT_ERR_ARG;
  if (!f || !io) return fail(c, LT_ERR_ARG, "null argument%s");
  return index_apply_impl(c, f, io, (hipStream_t)stream_);
}

static int index_apply_impl(lt_ctx* c, const lt_index* f, const lt_index_io* io,
                            hipStream_t stream_) {
  if (io->n_pix < 0 || io->n_obs < 0 || io->n_obs > 65535) return fail(c, LT_ERR_ARG, "bad sizes%s");
  if (io->n_pix == 0 || io->n_obs == 0) return LT_OK;
  if (!io->bands || !io->out) return fail(c, LT_ERR_ARG, "null buffer%s");
  // planar (pixel stride 1 or 0) or pixel-interleaved (band stride 1, pixel stride n_bands)
  const bool inter = io->band_pix_stride > 1;
  if (inter ? (io->band_pix_stride != f->n_bands || io->band_stride != 1 ||
               io->obs_stride < (int64_t)f->n_bands * io->n_pix)
            : (io->band_pix_stride < 0 || io->band_stride < io->n_pix ||
               io->obs_stride < (int64_t)f->n_bands * io->band_stride))
    return fail(c, LT_ERR_ARG, "bad strides%s");
  if (io->out_stride < io->n_pix) return fail(c, LT_ERR_ARG, "bad strides%s");
  HIP_OR_FAIL(c, hipSetDevice(c->device));
  long long obs_stride = io->obs_stride, band_stride = io->band_stride,
            out_stride = io->out_stride, pix_stride = inter ? io->band_pix_stride : 1;
  const size_t bsz = lt_idx::type_size(f->band_type), osz = lt_idx::type_size(f->out_type);
  // 4-pixel vector kernel over the 4-aligned head when every plane start is 4-element aligned
  const bool vec_ok = ((uintptr_t)io->bands % (4 * bsz)) == 0 &&
                      ((uintptr_t)io->out % (4 * osz)) == 0 && obs_stride % 4 == 0 &&
                      (inter || band_stride % 4 == 0) && out_stride % 4 == 0;
  const long long head = vec_ok ? (io->n_pix & ~3LL) : 0;
  if (head > 0) {
    const void* bands = io->bands;
    void* outp = io->out;
    long long n_pix = head;
    const unsigned gx = (unsigned)((head / 4 + 255) / 256);
    if (inter) {
      void* args[] = {(void*)&bands, &obs_stride, &n_pix, &outp, &out_stride};
      HIP_OR_FAIL(c, hipModuleLaunchKernel(f->fn4i, gx, (unsigned)io->n_obs, 1, 256, 1, 1, 0,
                                           (hipStream_t)stream_, args, nullptr));
    } else {
      void* args[] = {(void*)&bands, &obs_stride, &band_stride, &n_pix, &outp, &out_stride};
      HIP_OR_FAIL(c, hipModuleLaunchKernel(f->fn4, gx, (unsigned)io->n_obs, 1, 256, 1, 1, 0,
                                           (hipStream_t)stream_, args, nullptr));
    }
  }
  if (head < io->n_pix) {
    const void* bands = (const char*)io->bands + head * pix_stride * bsz;
    void* outp = (char*)io->out + head * osz;
    long long n_pix = io->n_pix - head;
    void* args[] = {(void*)&bands, &obs_stride, &band_stride, &n_pix, &outp, &out_stride,
                    &pix_stride};
    const unsigned gx = (unsigned)((n_pix + 255) / 256);
    HIP_OR_FAIL(c, hipModuleLaunchKernel(f->fn, gx, (unsigned)io->n_obs, 1, 256, 1, 1, 0,
                                         (hipStream_t)stream_, args, nullptr));
  }
  return LT_OK;
}
