// lt_raster.h — output raster assembly on the GPU (output_reducer, mr_land_trendr_job.py:128-152,
// -> data2raster, utils.py:414-440): one output key's raster built from a plane the analyze stage
// left in HBM, so only the finished raster (1 byte per pixel in the reference's GDT_Byte mode)
// crosses PCIe instead of every f64 plane.
//
// data2raster, per key: holder = ones_like(template) * NODATA (numpy 1.x promotion: the template
// type, or the next signed type for an unsigned template — land_trendr_amd/raster.holder_dtype),
// holder[y_off, x_off] = float(value) for every grid point the reducer emitted the key for (numpy's
// cast: truncation toward zero into an integer holder), then array2raster(holder, ..., compress)
// whose 4th positional parameter is data_type, so GDAL converts the holder to GDT_Byte: NaN -> 0,
// floats rounded half up, everything saturated to 0..255 (GDAL absent here:
// parity-unpinned, the same rules raster.py restates on the host).
// A grid point emits the key when its selector holds: matched[r] != 0 for '<rule>_<field>', winner
// [y] == obs id for 'trendline/<date>-<attr>'. Offsets must be unique (one grid point per pixel):
// the reference's loop lets the last duplicate win, an order a parallel scatter does not have, so
// the host checks uniqueness and assembles duplicated grids itself.
#pragma once
#include <stdint.h>

#include "../../include/lt_abi.h"

namespace lt {

// numpy float64 -> integer holder: x86 cvttsd2si into int64 (NaN / out of range -> INT64_MIN),
// then the two's-complement wrap of .astype(holder type)
__device__ inline int64_t np_f64_to_i64(double v) {
  if (!(v > -9223372036854775808.0 && v < 9223372036854775808.0)) return INT64_MIN;
  return (int64_t)v;  // truncation toward zero
}

// GDAL's GDT_Byte conversion of a holder value
__device__ inline uint8_t gdal_byte_i(int64_t h) { return (uint8_t)(h < 0 ? 0 : h > 255 ? 255 : h); }
__device__ inline uint8_t gdal_byte_f(double a) {
  if (a != a) return 0;
  const double r = __builtin_floor(a + 0.5);
  return (uint8_t)(r < 0.0 ? 0.0 : r > 255.0 ? 255.0 : r);
}
__device__ inline uint8_t gdal_byte_f32(float a) {
  if (a != a) return 0;
  const float r = __builtin_floorf(a + 0.5f);
  return (uint8_t)(r < 0.f ? 0.f : r > 255.f ? 255.f : r);
}

// the holder value of float(value) after the numpy cast into holder_type, as GDT_Byte
__device__ inline uint8_t holder_byte(double v, int holder_type) {
  switch (holder_type) {
    case LT_T_F64: return gdal_byte_f(v);
    case LT_T_F32: return gdal_byte_f32((float)v);
    case LT_T_I8: return gdal_byte_i((int8_t)np_f64_to_i64(v));
    case LT_T_I16: return gdal_byte_i((int16_t)np_f64_to_i64(v));
    case LT_T_I32: return gdal_byte_i((int32_t)np_f64_to_i64(v));
    case LT_T_U8: return gdal_byte_i((uint8_t)np_f64_to_i64(v));
    case LT_T_U16: return gdal_byte_i((uint16_t)np_f64_to_i64(v));
    case LT_T_U32: return gdal_byte_i((uint32_t)np_f64_to_i64(v));
    default: return gdal_byte_i(np_f64_to_i64(v));  // LT_T_I64
  }
}

__device__ inline double plane_value(const void* p, int t, int64_t i) {
  switch (t) {
    case LT_T_I32: return (double)((const int32_t*)p)[i];
    case LT_T_U8: return (double)((const uint8_t*)p)[i];
    case LT_T_I16: return (double)((const int16_t*)p)[i];
    default: return ((const double*)p)[i];
  }
}

// one output pixel's value for grid point p under job J (sel = the selector held)
__device__ inline void raster_store(const lt_raster_job& J, int64_t o, double v) {
  if (J.mode == LT_RASTER_REFERENCE) {
    ((uint8_t*)J.out)[o] = holder_byte(v, J.holder_type);
    return;
  }
  switch (J.out_type) {
    case LT_T_I32: ((int32_t*)J.out)[o] = (int32_t)v; break;
    case LT_T_U8: ((uint8_t*)J.out)[o] = (uint8_t)(int32_t)v; break;
    default: ((double*)J.out)[o] = v;
  }
}

__device__ inline bool raster_selected(const lt_raster_job& J, int64_t p) {
  if (J.sel_kind == LT_SEL_NONZERO) return ((const uint8_t*)J.sel)[p] != 0;
  if (J.sel_kind == LT_SEL_EQUALS) return ((const int16_t*)J.sel)[p] == J.sel_value;
  return true;
}

}  // namespace lt
