// lt_abi.hip — the C ABI of include/lt_abi.h: contexts, argument checks, scene upload, launches.
//
// Replaces, per pixel tile, the per-grid-point loop of MRLandTrendrJob.analysis_reducer
// (/root/reference/mr_land_trendr_job.py:83-126) around utils.analyze + utils.change_labeling.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/lt_abi.h"
#include "lt_pixel.h"

namespace {

constexpr int kBlock = 256;

template <int MAXY>
__global__ __launch_bounds__(kBlock) void analyze_kernel(const lt::DevScene* __restrict__ S,
                                                         const lt_params P, const lt_tile_in in,
                                                         const lt_tile_out out) {
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= in.n_pix) return;
  lt::analyze_pixel<MAXY>(*S, P, in, out, p);
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

}  // namespace

struct lt_ctx {
  int device = 0;
  std::string err;
  lt::DevScene* h_scene = nullptr;  // pinned staging
  lt::DevScene* d_scene = nullptr;
  hipEvent_t scene_copied = nullptr;
  bool scene_valid = false;
  bool timing = false;
  std::vector<EventPair> pool;   // all events ever created (reused)
  size_t used = 0;               // pairs recorded since the last stage_ms call
  double acc_ms = 0.0;
  int64_t launches = 0;
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

int lt_ctx_create(int device, lt_ctx** out) {
  if (!out) return LT_ERR_ARG;
  *out = nullptr;
  lt_ctx* c = new lt_ctx();
  c->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipHostMalloc((void**)&c->h_scene, sizeof(lt::DevScene));
  if (e == hipSuccess) e = hipMalloc((void**)&c->d_scene, sizeof(lt::DevScene));
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->scene_copied, hipEventDisableTiming);
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
  if (c->d_scene) (void)hipFree(c->d_scene);
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
  double acc = c->acc_ms;
  for (size_t i = 0; i < c->used; i++) {
    HIP_OR_FAIL(c, hipEventSynchronize(c->pool[i].stop));
    float ms = 0.f;
    HIP_OR_FAIL(c, hipEventElapsedTime(&ms, c->pool[i].start, c->pool[i].stop));
    acc += ms;
  }
  for (int s = 0; s < n_stages; s++) ms_out[s] = 0.0;
  if (n_stages > 1) ms_out[1] = acc;  // stage 1: fused winner+analyze+label kernel
  else if (n_stages == 1) ms_out[0] = acc;
  if (n_launches) *n_launches = c->launches;
  c->used = 0;
  c->acc_ms = 0.0;
  c->launches = 0;
  return LT_OK;
}

int lt_analyze_tile(lt_ctx* c, const lt_scene* sc, const lt_params* prm, const lt_tile_in* in,
                    const lt_tile_out* out, void* stream_) {
  if (!c) return LT_ERR_ARG;
  if (!sc || !prm || !in || !out) return fail(c, LT_ERR_ARG, "null argument%s");
  if (in->n_pix < 0 || in->stride < in->n_pix || out->stride < in->n_pix)
    return fail(c, LT_ERR_ARG, "bad n_pix/stride%s");
  if (in->n_pix == 0) return LT_OK;
  if (!in->obs_val) return fail(c, LT_ERR_ARG, "obs_val is required%s");
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
  HIP_OR_FAIL(c, hipSetDevice(c->device));
  hipStream_t stream = (hipStream_t)stream_;

  // scene upload (skipped when identical to the resident one)
  lt::DevScene tmp;
  memset(&tmp, 0, sizeof tmp);
  tmp.n_obs = K;
  tmp.n_years = Y;
  for (int y = 0; y < Y; y++) {
    tmp.year[y] = sc->year[y];
    tmp.feb29_bad[y] = sc->feb29_bad ? sc->feb29_bad[y] : 0;
  }
  for (int y = 0; y <= Y; y++) tmp.slot_begin[y] = Y > 0 ? sc->slot_begin[y] : 0;
  for (int k = 0; k < K; k++) {
    tmp.order[k] = sc->order[k];
    tmp.dist[k] = sc->dist[k];
  }
  if (!c->scene_valid || memcmp(&tmp, c->h_scene, sizeof tmp) != 0) {
    HIP_OR_FAIL(c, hipEventSynchronize(c->scene_copied));  // staging buffer free again
    memcpy(c->h_scene, &tmp, sizeof tmp);
    HIP_OR_FAIL(c, hipMemcpyAsync(c->d_scene, c->h_scene, sizeof tmp, hipMemcpyHostToDevice,
                                  stream));
    HIP_OR_FAIL(c, hipEventRecord(c->scene_copied, stream));
    c->scene_valid = true;
  }

  EventPair* ep = nullptr;
  if (c->timing) {
    if (c->used == c->pool.size()) {
      EventPair np;
      HIP_OR_FAIL(c, hipEventCreate(&np.start));
      HIP_OR_FAIL(c, hipEventCreate(&np.stop));
      c->pool.push_back(np);
    }
    ep = &c->pool[c->used++];
    HIP_OR_FAIL(c, hipEventRecord(ep->start, stream));
  }
  const int64_t nblk = (in->n_pix + kBlock - 1) / kBlock;
  if (nblk > 0x7fffffff) return fail(c, LT_ERR_LIMIT, "tile too large%s");
  dim3 grid((unsigned)nblk), block(kBlock);
  if (Y <= 32)
    hipLaunchKernelGGL(analyze_kernel<32>, grid, block, 0, stream, c->d_scene, *prm, *in, *out);
  else
    hipLaunchKernelGGL(analyze_kernel<64>, grid, block, 0, stream, c->d_scene, *prm, *in, *out);
  HIP_OR_FAIL(c, hipGetLastError());
  if (ep) HIP_OR_FAIL(c, hipEventRecord(ep->stop, stream));
  c->launches++;
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

}  // extern "C"
