// lt_index.h — the load stage (settings.json index_eqn, utils.py:447-484 rast_algebra) as a kernel
// generated per equation and compiled at run time with hiprtc. Included by lt_abi.hip (host code).
//
// The host (land_trendr_amd/index_eqn.py) turns the equation into a typed postfix program with
// numpy 1.x semantics; here the program becomes straight-line HIP source (one SSA value per
// node), so the kernel is a single streaming pass: n_bands loads, a handful of VALU ops and one
// store per observation-pixel, no interpretation. The source is generated from the validated
// program only — never from equation text.
#pragma once
#include <hip/hiprtc.h>

#include <cmath>
#include <map>
#include <string>
#include <vector>

struct lt_index {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr, fn4 = nullptr, fn4i = nullptr;
  int32_t n_bands = 0, band_type = 0, out_type = 0;
  lt_index_prog prog{};  // the program (JIT analyze kernels inline it, lt_jit.h)
};

namespace lt_idx {

inline const char* ctype(int t) {
  switch (t) {
    case LT_T_F64: return "double";
    case LT_T_I16: return "short";
    case LT_T_U16: return "unsigned short";
    case LT_T_I32: return "int";
    case LT_T_F32: return "float";
    case LT_T_U8: return "unsigned char";
    case LT_T_U32: return "unsigned int";
    case LT_T_I8: return "signed char";
    case LT_T_I64: return "long long";
    default: return nullptr;
  }
}
inline bool is_float(int t) { return t == LT_T_F64 || t == LT_T_F32; }
inline size_t type_size(int t) {
  switch (t) {
    case LT_T_F64: case LT_T_I64: return 8;
    case LT_T_I32: case LT_T_F32: case LT_T_U32: return 4;
    case LT_T_I16: case LT_T_U16: return 2;
    default: return 1;
  }
}
inline bool is_unsigned(int t) { return t == LT_T_U16 || t == LT_T_U8 || t == LT_T_U32; }
// integer range of a type (for the saturating store)
inline void int_range(int t, long long& lo, long long& hi) {
  switch (t) {
    case LT_T_I16: lo = -32768; hi = 32767; break;
    case LT_T_U16: lo = 0; hi = 65535; break;
    case LT_T_I32: lo = -2147483647LL - 1; hi = 2147483647LL; break;
    case LT_T_U8: lo = 0; hi = 255; break;
    case LT_T_U32: lo = 0; hi = 4294967295LL; break;
    case LT_T_I8: lo = -128; hi = 127; break;
    default: lo = -9223372036854775807LL - 1; hi = 9223372036854775807LL; break;
  }
}

// Device helpers every generated kernel carries (numpy's integer and float loops).
constexpr const char* kPrelude = R"HIP(
// integer floor division with numpy's rules: floor (Python), x / 0 -> 0
__device__ static inline long long lt_ifloordiv(long long a, long long b) {
  if (b == 0) return 0;
  if (a == (-9223372036854775807LL - 1) && b == -1) return a;
  long long q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) q -= 1;
  return q;
}
__device__ static inline unsigned long long lt_ufloordiv(unsigned long long a,
                                                         unsigned long long b) {
  return b == 0 ? 0ull : a / b;
}
// numpy npy_divmod's floor division for floating point
template <class F>
__device__ static inline F lt_ffloordiv(F a, F b) {
  if (b == (F)0) return a / b;
  F mod = fmod(a, b);
  F div = (a - mod) / b;
  if (mod != (F)0) {
    if ((b < (F)0) != (mod < (F)0)) div -= (F)1;
  }
  F fd;
  if (div != (F)0) {
    fd = floor(div);
    if (div - fd > (F)0.5) fd += (F)1;
  } else {
    fd = copysign((F)0, a / b);
  }
  return fd;
}
)HIP";

struct Val {
  std::string name;
  int type;
};

// expression of value v converted to type t (numpy casts every operand to the node's type)
inline std::string cast_to(const Val& v, int t) {
  if (v.type == t) return v.name;
  return std::string("((") + ctype(t) + ")" + v.name + ")";
}

inline std::string fmt_double(double d) {
  char b[64];
  snprintf(b, sizeof b, "%a", d);
  return b;
}

// Generated source for prog, or "" with err set. Three kernels: lt_index_kernel (one pixel per
// thread, any pixel stride), lt_index_kernel4 (four consecutive pixels per thread, vector loads
// and stores, for 4-aligned planar bands) and lt_index_kernel4i (the same for pixel-interleaved
// bands); the host sends the tail to the scalar one.
inline std::string codegen_body(const lt_index_prog& P, bool vec, std::string& err,
                                std::string& store_out);
inline std::string codegen(const lt_index_prog& P, std::string& err) {
  std::string store1, store4;
  const std::string body1 = codegen_body(P, false, err, store1);
  if (body1.empty()) return "";
  const std::string body4 = codegen_body(P, true, err, store4);
  const char* BT = ctype(P.band_type);
  const char* OT = ctype(P.out_type);
  std::string src = kPrelude;
  src += std::string("typedef ") + BT + " lt_bt4 __attribute__((ext_vector_type(4)));\n";
  src += std::string("typedef ") + OT + " lt_ot4 __attribute__((ext_vector_type(4)));\n";
  src += std::string("extern \"C\" __global__ __launch_bounds__(256) void lt_index_kernel(const ") +
         BT + "* __restrict__ bands, long long obs_stride, long long band_stride, long long n_pix, " +
         OT + "* __restrict__ out, long long out_stride, long long pix_stride) {\n"
         "  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;\n"
         "  const long long o = blockIdx.y;\n"
         "  if (p >= n_pix) return;\n"
         "  const " + BT + "* b = bands + o * obs_stride + p * pix_stride;\n";
  src += body1;
  src += "  out[o * out_stride + p] = " + store1 + ";\n}\n";
  src += std::string("extern \"C\" __global__ __launch_bounds__(256) void lt_index_kernel4(const ") +
         BT + "* __restrict__ bands, long long obs_stride, long long band_stride, long long n_pix, " +
         OT + "* __restrict__ out, long long out_stride) {\n"
         "  const long long p = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;\n"
         "  const long long o = blockIdx.y;\n"
         "  if (p >= n_pix) return;\n"
         "  const " + BT + "* b = bands + o * obs_stride + p;\n";
  for (int s = 0; s < P.n_bands; s++)
    src += "  const lt_bt4 bv" + std::to_string(s) + " = *(const lt_bt4*)(b + " +
           std::to_string(s) + "LL * band_stride);\n";
  src += "  lt_ot4 res;\n#pragma unroll\n  for (int j = 0; j < 4; j++) {\n";
  src += body4;
  src += "  res[j] = " + store4 + ";\n  }\n  *(lt_ot4*)(out + o * out_stride + p) = res;\n}\n";
  // pixel-interleaved bands (band s of pixel p at p * n_bands + s): a 4-pixel group's n_bands * 4
  // values are contiguous, read as n_bands 4-element vector loads and regrouped per band
  const int nb = P.n_bands;
  src += std::string("extern \"C\" __global__ __launch_bounds__(256) void lt_index_kernel4i(const ") +
         BT + "* __restrict__ bands, long long obs_stride, long long n_pix, " + OT +
         "* __restrict__ out, long long out_stride) {\n"
         "  const long long p = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;\n"
         "  const long long o = blockIdx.y;\n"
         "  if (p >= n_pix) return;\n"
         "  const " + BT + "* b = bands + o * obs_stride + p * " + std::to_string(nb) + "LL;\n";
  for (int k = 0; k < nb; k++)
    src += "  const lt_bt4 c" + std::to_string(k) + " = *(const lt_bt4*)(b + " +
           std::to_string(4 * k) + ");\n";
  for (int sb = 0; sb < nb; sb++) {
    src += "  lt_bt4 bv" + std::to_string(sb) + ";\n";
    for (int j = 0; j < 4; j++) {
      const int e = j * nb + sb;
      src += "  bv" + std::to_string(sb) + "[" + std::to_string(j) + "] = c" +
             std::to_string(e / 4) + "[" + std::to_string(e % 4) + "];\n";
    }
  }
  src += "  lt_ot4 res;\n#pragma unroll\n  for (int j = 0; j < 4; j++) {\n";
  src += body4;
  src += "  res[j] = " + store4 + ";\n  }\n  *(lt_ot4*)(out + o * out_stride + p) = res;\n}\n";
  return src;
}

inline std::string codegen_body(const lt_index_prog& P, bool vec, std::string& err,
                                std::string& store_out) {
  if (P.n_ops < 1 || P.n_ops > LT_MAX_PROG || P.n_bands < 1 || P.n_bands > LT_MAX_BANDS ||
      !ctype(P.band_type) || !ctype(P.out_type)) {
    err = "index program: bad sizes or types";
    return "";
  }
  std::string body;
  std::vector<Val> st;
  char line[512];
  for (int k = 0; k < P.n_ops; k++) {
    const lt_index_op& o = P.ops[k];
    const std::string v = "v" + std::to_string(k);
    if (!ctype(o.type)) {
      err = "index program: bad node type";
      return "";
    }
    const char* T = ctype(o.type);
    switch (o.op) {
      case LT_OP_BAND:
        if (o.ival < 0 || o.ival >= P.n_bands || o.type != P.band_type) {
          err = "index program: bad band slot";
          return "";
        }
        if (vec)
          snprintf(line, sizeof line, "  const %s %s = bv%lld[j];\n", T, v.c_str(),
                   (long long)o.ival);
        else
          snprintf(line, sizeof line, "  const %s %s = b[%lldLL * band_stride];\n", T, v.c_str(),
                   (long long)o.ival);
        body += line;
        st.push_back({v, o.type});
        break;
      case LT_OP_CONST_I:
        snprintf(line, sizeof line, "  const long long %s = %lldLL;\n", v.c_str(),
                 (long long)o.ival);
        body += line;
        st.push_back({v, LT_T_I64});
        break;
      case LT_OP_CONST_F:
        if (!std::isfinite(o.fval)) {
          err = "index program: non-finite constant";
          return "";
        }
        body += "  const double " + v + " = " + fmt_double(o.fval) + ";\n";
        st.push_back({v, LT_T_F64});
        break;
      case LT_OP_NEG: {
        if (st.empty()) {
          err = "index program: stack underflow";
          return "";
        }
        Val a = st.back();
        st.pop_back();
        std::string e;
        if (is_float(o.type))
          e = "-" + cast_to(a, o.type);
        else  // two's complement wrap
          e = std::string("(") + T + ")(0ull - (unsigned long long)" + cast_to(a, o.type) + ")";
        body += std::string("  const ") + T + " " + v + " = " + e + ";\n";
        st.push_back({v, o.type});
        break;
      }
      case LT_OP_ADD:
      case LT_OP_SUB:
      case LT_OP_MUL:
      case LT_OP_DIV:
      case LT_OP_FLOORDIV: {
        if (st.size() < 2) {
          err = "index program: stack underflow";
          return "";
        }
        Val b = st.back();
        st.pop_back();
        Val a = st.back();
        st.pop_back();
        const std::string x = cast_to(a, o.type), y = cast_to(b, o.type);
        std::string e;
        if (is_float(o.type)) {
          if (o.op == LT_OP_FLOORDIV)
            e = std::string("lt_ffloordiv<") + T + ">(" + x + ", " + y + ")";
          else
            e = x + (o.op == LT_OP_ADD ? " + " : o.op == LT_OP_SUB ? " - " : o.op == LT_OP_MUL ? " * " : " / ") + y;
        } else if (o.op == LT_OP_DIV || o.op == LT_OP_FLOORDIV) {
          e = is_unsigned(o.type)
                  ? std::string("(") + T + ")lt_ufloordiv((unsigned long long)" + x +
                        ", (unsigned long long)" + y + ")"
                  : std::string("(") + T + ")lt_ifloordiv((long long)" + x + ", (long long)" +
                        y + ")";
        } else {  // wrap: the exact result modulo 2^bits
          const char* opc = o.op == LT_OP_ADD ? " + " : o.op == LT_OP_SUB ? " - " : " * ";
          e = std::string("(") + T + ")((unsigned long long)(long long)" + x + opc +
              "(unsigned long long)(long long)" + y + ")";
        }
        body += std::string("  const ") + T + " " + v + " = " + e + ";\n";
        st.push_back({v, o.type});
        break;
      }
      default:
        err = "index program: bad opcode";
        return "";
    }
  }
  if (st.size() != 1) {
    err = "index program: stack not balanced";
    return "";
  }
  // the store into the template's type (GDAL's conversion; parity-unpinned, index_eqn.py)
  const Val r = st.back();
  const char* OT = ctype(P.out_type);
  std::string store;
  if (r.type == P.out_type) {
    store = r.name;
  } else if (is_float(P.out_type)) {
    store = std::string("(") + OT + ")" + r.name;
  } else {
    long long lo, hi;
    int_range(P.out_type, lo, hi);
    char b[256];
    if (is_float(r.type)) {
      snprintf(b, sizeof b,
               "(%s)(%s != %s ? 0.0 : fmin(fmax(floor((double)%s + 0.5), %lld.0), %lld.0))", OT,
               r.name.c_str(), r.name.c_str(), r.name.c_str(), lo, hi);
    } else if (is_unsigned(r.type)) {
      snprintf(b, sizeof b, "(%s)((unsigned long long)%s > %lldull ? %lldull : "
               "(unsigned long long)%s)", OT, r.name.c_str(), hi, hi, r.name.c_str());
    } else {
      snprintf(b, sizeof b, "(%s)((long long)%s < %lldLL ? %lldLL : (long long)%s > %lldLL ? "
               "%lldLL : (long long)%s)", OT, r.name.c_str(), lo, lo, r.name.c_str(), hi, hi,
               r.name.c_str());
    }
    store = b;
  }
  store_out = store;
  return body;
}

inline bool is_int(int t) { return ctype(t) && !is_float(t); }

// A program's integer linear form (lt_abi.h lt_index_lin), or false. Every arithmetic node must
// carry the one integer type W (numpy wraps each node modulo 2^bits(W), so the whole sum taken
// modulo 2^64 and wrapped once at the end is the same value); band operands are cast to W, which
// must hold every band value; integer constants are cast to W by wrapping, which the modular sum
// absorbs; a product needs a constant side; no division and no float node.
inline bool linearize(const lt_index_prog& P, lt_index_lin& L) {
  L = lt_index_lin{};
  if (P.n_ops < 1 || P.n_ops > LT_MAX_PROG || P.n_bands < 1 || P.n_bands > LT_LIN_MAX_BANDS)
    return false;
  const int bt = P.band_type;
  if (bt != LT_T_I16 && bt != LT_T_U16 && bt != LT_T_U8 && bt != LT_T_I32) return false;
  if (!ctype(P.out_type)) return false;
  struct Form {
    bool band;  // some coefficient may be non-zero (a band term)
    uint64_t c0, c[LT_LIN_MAX_BANDS];
  };
  std::vector<Form> st;
  int W = -1;
  // a band of type bt cast to W keeps its value
  auto holds = [&](int w) {
    long long blo, bhi, wlo, whi;
    int_range(bt, blo, bhi);
    int_range(w, wlo, whi);
    if (w == LT_T_U32 && bt == LT_T_I32) return false;
    return blo >= wlo && bhi <= whi;
  };
  for (int k = 0; k < P.n_ops; k++) {
    const lt_index_op& o = P.ops[k];
    Form f{};
    switch (o.op) {
      case LT_OP_BAND:
        if (o.ival < 0 || o.ival >= P.n_bands || o.type != bt) return false;
        f.band = true;
        f.c[o.ival] = 1;
        st.push_back(f);
        continue;
      case LT_OP_CONST_I:
        f.c0 = (uint64_t)o.ival;
        st.push_back(f);
        continue;
      case LT_OP_ADD:
      case LT_OP_SUB:
      case LT_OP_MUL:
      case LT_OP_NEG:
        break;
      default:  // a float constant, a division
        return false;
    }
    if (!is_int(o.type) || (W >= 0 && o.type != W)) return false;
    W = o.type;
    if (o.op == LT_OP_NEG) {
      if (st.empty()) return false;
      Form& a = st.back();
      a.c0 = 0 - a.c0;
      for (int s = 0; s < LT_LIN_MAX_BANDS; s++) a.c[s] = 0 - a.c[s];
      continue;
    }
    if (st.size() < 2) return false;
    const Form b = st.back();
    st.pop_back();
    Form& a = st.back();
    if (o.op == LT_OP_MUL) {
      if (a.band && b.band) return false;  // a product of two band terms
      const Form& cst = a.band ? b : a;
      const Form& var = a.band ? a : b;
      Form r{};
      r.band = var.band;
      r.c0 = var.c0 * cst.c0;
      for (int s = 0; s < LT_LIN_MAX_BANDS; s++) r.c[s] = var.c[s] * cst.c0;
      a = r;
    } else {
      const bool sub = o.op == LT_OP_SUB;
      a.band = a.band || b.band;
      a.c0 = sub ? a.c0 - b.c0 : a.c0 + b.c0;
      for (int s = 0; s < LT_LIN_MAX_BANDS; s++) a.c[s] = sub ? a.c[s] - b.c[s] : a.c[s] + b.c[s];
    }
  }
  if (st.size() != 1) return false;
  if (W < 0) W = bt;  // the program is one band plane: its values, stored into out_type
  if (!holds(W)) return false;
  L.n_bands = P.n_bands;
  L.band_type = bt;
  L.wrap_type = W;
  L.out_type = P.out_type;
  L.c0 = (int64_t)st[0].c0;
  for (int s = 0; s < LT_LIN_MAX_BANDS; s++) L.coef[s] = (int64_t)st[0].c[s];
  return true;
}

}  // namespace lt_idx
