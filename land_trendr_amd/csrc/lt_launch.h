// lt_launch.h — what lt_abi.hip hands the analyze-stage dispatch for one tile.
//
// The kernels of the analyze and resolve stages (lt_kernels.h) are instantiated in a dispatch
// translation unit of their own: lt_dispatch.hip in the product library, a profiling unit in the
// profiling builds (profiles/). lt_abi.hip (contexts, argument checks, scene upload, streams,
// events) only sees this record and the two entry points below.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lt_abi.h"
#include "lt_pixel.h"

namespace lt {

struct TileLaunch {
  const DevScene* scene;         // device copy of the tile's scene
  const lt_params* params;       // host struct (passed by value to the kernels)
  const lt_tile_in* in;
  const lt_tile_out* out;
  const lsq_xf* xtab;            // the context's x-set factor table
  int64_t* defer;                // [2][n_pix]: the binary32 and the binary64 deferred lists
  unsigned long long* counters;  // [4]: list counts [0]/[2], resolve work counters [1]/[3]
  uint64_t* yflags;              // [2][n_pix] spike / vertex year flags, or null
  int n_years;                   // Y
  int device;
  hipStream_t stream;
  uint64_t* tl_bits = nullptr;   // the compact trendline ([4][n_pix] words), or null
  double* tl_eqn = nullptr;      // its segment eqns ([Y-1][n_pix] (m, b) pairs)
};

// Stage 1: the analyze kernel over every pixel of the tile, on l.stream.
hipError_t launch_analyze(const TileLaunch& l);
// Stage 2: the resolve kernels over the pixels stage 1 deferred, on l.stream.
hipError_t launch_resolve(const TileLaunch& l);

}  // namespace lt
