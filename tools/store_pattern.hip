// store_pattern.hip — the HBM write rate of the c5 output layout (per-year planes [Y][P], binary64
// and u8) for the store patterns a kernel can use, with no arithmetic: what bounds the year-major
// loop of the analyze kernel (one 64-pixel wave, 512 B per binary64 row piece) and the streaming
// expand kernel (lt_abi.hip trendline_expand_kernel), against one flat buffer of the same size.
// Each pattern writes F binary64 planes (+ U u8 planes) of Y rows x P pixels; kernel time by HIP
// events, best of R repetitions. Prints one JSON object.
//   flat          one contiguous buffer of the same bytes, 16 B per lane, grid-stride
//   wave64        one wave per workgroup, one pixel per lane, rows in (year, plane) order: the
//                 analyze kernel's year-major loop (512 B per row piece)
//   blk<N>        256-thread workgroups over N consecutive pixels (N/256 per thread, 256-strided),
//                 rows in (year, plane) order: N*8 B contiguous per row piece
//   rowmajor      each workgroup fills one 32 KB piece of one row; pieces of a row consecutive
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

struct Planes {
  double* f[8];
  uint8_t* u[2];
  int nf, nu;
  int64_t P;
  int Y;
};

__global__ __launch_bounds__(256) void flat_kernel(double* __restrict__ b, int64_t n2, bool nt) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  d2* v = (d2*)b;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
    const d2 x = d2{(double)i, (double)(i + 1)};
    if (nt)
      __builtin_nontemporal_store(x, v + i);
    else
      v[i] = x;
  }
}

template <int WG>
__global__ __launch_bounds__(WG) void rows_kernel(const Planes pl, int ppt, bool nt) {
  const int64_t base = (int64_t)blockIdx.x * WG * ppt;
  for (int y = 0; y < pl.Y; y++) {
    const int64_t row = (int64_t)y * pl.P;
    for (int f = 0; f < pl.nf; f++)
      for (int j = 0; j < ppt; j++) {
        const int64_t p = base + j * WG + threadIdx.x;
        if (p >= pl.P) break;
        const double x = (double)(p + y + f);
        if (nt)
          __builtin_nontemporal_store(x, pl.f[f] + row + p);
        else
          pl.f[f][row + p] = x;
      }
    for (int f = 0; f < pl.nu; f++)
      for (int j = 0; j < ppt; j++) {
        const int64_t p = base + j * WG + threadIdx.x;
        if (p >= pl.P) break;
        pl.u[f][row + p] = (uint8_t)(p + y);
      }
  }
}

// one workgroup per (row, 4096-pixel piece), pieces of one row consecutive
__global__ __launch_bounds__(256) void rowmajor_kernel(const Planes pl, bool nt) {
  const int64_t pieces = (pl.P + 4095) / 4096;
  const int64_t r = blockIdx.x / pieces, c = blockIdx.x % pieces;
  const int y = (int)(r / (pl.nf + pl.nu)), f = (int)(r % (pl.nf + pl.nu));
  const int64_t row = (int64_t)y * pl.P;
  for (int j = 0; j < 16; j++) {
    const int64_t p = c * 4096 + j * 256 + threadIdx.x;
    if (p >= pl.P) break;
    if (f < pl.nf) {
      const double x = (double)(p + y + f);
      if (nt)
        __builtin_nontemporal_store(x, pl.f[f] + row + p);
      else
        pl.f[f][row + p] = x;
    } else {
      pl.u[f - pl.nf][row + p] = (uint8_t)(p + y);
    }
  }
}

int main(int argc, char** argv) {
  const int64_t P = argc > 1 ? atoll(argv[1]) : (1ll << 24);
  const int Y = argc > 2 ? atoi(argv[2]) : 40;
  const int NF = argc > 3 ? atoi(argv[3]) : 5;
  const int NU = argc > 4 ? atoi(argv[4]) : 2;
  const int R = 5;
  Planes pl;
  pl.nf = NF;
  pl.nu = NU;
  pl.P = P;
  pl.Y = Y;
  for (int f = 0; f < NF; f++) CK(hipMalloc(&pl.f[f], (size_t)P * Y * 8));
  for (int f = 0; f < NU; f++) CK(hipMalloc(&pl.u[f], (size_t)P * Y));
  const double bytes = (double)P * Y * (8.0 * NF + NU);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto launch) {
    float best = 1e30f;
    for (int r = 0; r < R; r++) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    CK(hipGetLastError());
    return best;
  };
  std::string js = "{\"pixels\": " + std::to_string(P) + ", \"years\": " + std::to_string(Y) +
                   ", \"f64_planes\": " + std::to_string(NF) + ", \"u8_planes\": " +
                   std::to_string(NU) + ", \"bytes\": " + std::to_string(bytes) +
                   ", \"best_of\": " + std::to_string(R) + ", \"patterns\": {";
  bool first = true;
  auto add = [&](const std::string& name, float ms, double b) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s\"%s\": {\"ms\": %.4f, \"TB_s\": %.3f}", first ? "" : ", ",
             name.c_str(), ms, b / (ms * 1e-3) / 1e12);
    js += buf;
    first = false;
    fprintf(stderr, "%s %.3f ms %.3f TB/s\n", name.c_str(), ms, b / (ms * 1e-3) / 1e12);
  };
  // flat: the f64 bytes as one buffer (the first plane's allocation is P*Y*8; use all planes' sum
  // by writing plane 0..NF-1 in turn, each contiguous)
  for (int nt = 0; nt < 2; nt++) {
    const float ms = timeit([&] {
      for (int f = 0; f < NF; f++)
        hipLaunchKernelGGL(flat_kernel, dim3(8192), dim3(256), 0, 0, pl.f[f], P * Y / 2, nt != 0);
    });
    add(std::string("flat_f64") + (nt ? "_nt" : ""), ms, (double)P * Y * 8.0 * NF);
  }
  for (int nt = 0; nt < 2; nt++) {
    const float ms = timeit([&] {
      hipLaunchKernelGGL(rows_kernel<64>, dim3((unsigned)((P + 63) / 64)), dim3(64), 0, 0, pl, 1,
                         nt != 0);
    });
    add(std::string("wave64") + (nt ? "_nt" : ""), ms, bytes);
  }
  for (int ppt : {1, 2, 4, 8, 16}) {
    for (int nt = 0; nt < 2; nt++) {
      const int64_t per = 256ll * ppt;
      const float ms = timeit([&] {
        hipLaunchKernelGGL(rows_kernel<256>, dim3((unsigned)((P + per - 1) / per)), dim3(256), 0,
                           0, pl, ppt, nt != 0);
      });
      add("blk" + std::to_string(per) + (nt ? "_nt" : ""), ms, bytes);
    }
  }
  for (int nt = 0; nt < 2; nt++) {
    const int64_t pieces = (P + 4095) / 4096;
    const float ms = timeit([&] {
      hipLaunchKernelGGL(rowmajor_kernel, dim3((unsigned)(pieces * Y * (NF + NU))), dim3(256), 0, 0,
                         pl, nt != 0);
    });
    add(std::string("rowmajor") + (nt ? "_nt" : ""), ms, bytes);
  }
  js += "}}";
  printf("%s\n", js.c_str());
  return 0;
}
