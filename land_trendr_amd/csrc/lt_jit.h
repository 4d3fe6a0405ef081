// lt_jit.h — analyze / resolve kernels JIT-specialised for one index_eqn program (host code,
// included by lt_abi.hip).
//
// The reference evaluates any index_eqn with Python 2 eval over band arrays, per raster
// (rast_algebra, /root/reference/utils.py:447-484), before apply_grid reads each pixel back
// (utils.py:357). An integer linear program ('B1 - B2') is folded into the precompiled analyze
// kernel (lt_index_lin). Any other program (divisions, float nodes, products of bands) is inlined
// here: the load kernel's straight-line code for the program (lt_index.h codegen: numpy 1.x typed
// arithmetic, Python 2 floor division, x / 0 = 0, the store into the index raster's type) becomes
// lt_jit_index(), and the analyze / resolve bodies of lt_kernels_dev.h are compiled around it with
// hiprtc (LT_JIT_INDEX in lt_fast.h's winner pick). No index raster is written and no load kernel
// runs between the analyze launches of consecutive tiles.
//
// One module per (program, MAXY, RMAX, series type), compiled on first use (~10 s per kernel)
// and cached in the context; the code object is also cached on disk (LT_JIT_CACHE, default
// <library dir>/../build/jit) under a hash of the generated source, the compile options and the
// kernel headers it includes, so later processes load it at once.
#pragma once
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "lt_index.h"
#include "lt_pixel.h"

struct lt_jit_kernels {
  hipModule_t mod = nullptr;
  hipFunction_t analyze = nullptr, resolve = nullptr, resolve64 = nullptr;
  unsigned resolve_grid = 0, resolve64_grid = 0;  // resident waves of each resolve kernel
};

namespace lt_jit {

// hiprtc carries no standard headers: the few names the kernel headers use from them
constexpr const char* kRtcPrelude = R"HIP(
typedef __hip_internal::int8_t int8_t;
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::int16_t int16_t;
typedef __hip_internal::uint16_t uint16_t;
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::int64_t int64_t;
typedef __hip_internal::uint64_t uint64_t;
typedef unsigned long uintptr_t;
#define INT32_MIN (-2147483647 - 1)
#define INT32_MAX 2147483647
namespace std {
using __hip_internal::false_type;
using __hip_internal::is_same;
using __hip_internal::true_type;
}
)HIP";

// the directory of the kernel headers: LT_SRC_DIR, else csrc/ beside this library
inline std::string src_dir() {
  const char* e = getenv("LT_SRC_DIR");
  if (e && *e) return e;
  Dl_info info;
  if (dladdr((void*)&src_dir, &info) && info.dli_fname) {
    std::string p = info.dli_fname;
    const size_t s = p.rfind('/');
    return (s == std::string::npos ? std::string(".") : p.substr(0, s)) + "/csrc";
  }
  return "csrc";
}

inline std::string cache_dir(const std::string& srcdir) {
  const char* e = getenv("LT_JIT_CACHE");
  if (e) return e;  // "" disables the disk cache
  return srcdir + "/../../build/jit";
}

inline bool read_file(const std::string& path, std::string& out) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  char buf[65536];
  size_t n;
  out.clear();
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, n);
  fclose(f);
  return true;
}

inline uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char ch : s) {
    h ^= ch;
    h *= 1099511628211ull;
  }
  return h;
}

// the series type of the analyze stage (lt_kernels.h series_kind): int16 for an int16 index,
// binary64 for a binary64 index with <= 4 rules, else binary32
inline const char* series_type(int out_type, int n_rules) {
  if (out_type == LT_T_I16) return "short";
  if (out_type == LT_T_F64 && n_rules <= 4) return "double";
  return "float";
}

// The launch-uniform values a module is specialised for (lt_fast.h LT_SPEC_*): the scene's year
// count, whether the tile has a cloud mask, whether any per-year plane is written, the rules, the
// pre_threshold mode and the line cost. Constant-folded, they remove the code of every other case
// (the mask scan, the year-major output loop or the labels-only paths, the rule filters).
struct Spec {
  bool on = false;
  int n_years = 0;
  bool masked = false, year_out = false;
  lt_params params{};
  const lt::DevScene* scene = nullptr;  // the scene's tables as constants (LT_SPEC_SCENE)
};

// a DevScene as a C++ initializer (the arrays up to their used length; the rest zero-fills)
inline std::string fmt_scene(const lt::DevScene& S) {
  std::string r = "{" + std::to_string(S.n_obs) + ", " + std::to_string(S.n_years) + ", " +
                  std::to_string((unsigned long long)S.feb29_mask) + "ull";
  auto arr = [&](const int32_t* a, int n) {
    r += ", {";
    for (int i = 0; i < n; i++) r += (i ? "," : "") + std::to_string(a[i]);
    r += "}";
  };
  arr(S.year, S.n_years);
  arr(S.slot_begin, S.n_years + 1);
  arr(S.order, S.n_obs);
  arr(S.dist, S.n_obs);
  arr(S.winner_all, S.n_years);
  return r + "}";
}

inline std::string fmt_rule(const lt_rule& r) {
  char b[256];
  snprintf(b, sizeof b, "{%d, %d, %d, %d, %a, %a, %a, %d, 0}", r.change_type, r.onset_op,
           r.duration_op, r.pre_op, r.onset_val, r.duration_val, r.pre_val, r.class_val);
  return b;
}

// The module source for program P, kernel instance (maxy, rmax), series type vt and
// specialisation sp; "" with err
inline std::string source(const lt_index_prog& P, int maxy, int rmax, const char* vt,
                          const Spec& sp, std::string& err) {
  std::string store;
  const std::string body = lt_idx::codegen_body(P, false, err, store);
  if (body.empty()) return "";
  const char* BT = lt_idx::ctype(P.band_type);
  char head[256];
  std::string src = kRtcPrelude;
  src += lt_idx::kPrelude;
  snprintf(head, sizeof head, "#define LT_JIT_INDEX 1\n#define LT_JIT_BAND_T %s\n", BT);
  src += head;
  // A/B runs: LT_JIT_DEFINES="NAME=VALUE,NAME2=VALUE2" adds compile-time switches of the kernel
  // headers (LT_RESOLVE_FULL, LT_WB, ...) to the generated source (and so to its cache key)
  if (const char* e = getenv("LT_JIT_DEFINES")) {
    std::string s(e);
    size_t at = 0;
    while (at < s.size()) {
      size_t end = s.find(',', at);
      if (end == std::string::npos) end = s.size();
      std::string d = s.substr(at, end - at);
      const size_t eq = d.find('=');
      if (!d.empty()) src += "#define " + (eq == std::string::npos ? d : d.substr(0, eq) + " " + d.substr(eq + 1)) + "\n";
      at = end + 1;
    }
  }
  if (sp.on) {
    const lt_params& Q = sp.params;
    char d[512];
    snprintf(d, sizeof d,
             "#include \"../../include/lt_abi.h\"\n#define LT_SPEC_Y %d\n#define LT_SPEC_MASKED %d\n"
             "#define LT_SPEC_YEAR_OUT %d\n#define LT_SPEC_NRULES %d\n#define LT_SPEC_PRE_MODE %d\n"
             "#define LT_SPEC_LINE_COST %a\n",
             sp.n_years, sp.masked ? 1 : 0, sp.year_out ? 1 : 0, Q.n_rules, Q.pre_threshold_mode,
             Q.line_cost);
    src += d;
    src += "__device__ constexpr lt_rule lt_spec_rules[" +
           std::to_string(Q.n_rules > 0 ? Q.n_rules : 1) + "] = {";
    for (int r = 0; r < (Q.n_rules > 0 ? Q.n_rules : 1); r++)
      src += (r ? ", " : "") + fmt_rule(Q.rules[r]);
    src += "};\n";
  }
  if (sp.on && sp.scene) {
    src += "#include \"lt_pixel.h\"\n#define LT_SPEC_SCENE 1\n";
    src += "__device__ constexpr lt::DevScene lt_spec_scene = " + fmt_scene(*sp.scene) + ";\n";
  }
  src += "__device__ inline double lt_jit_index(const LT_JIT_BAND_T* b, long long band_stride) {\n";
  src += body;
  src += "  return (double)(" + store + ");\n}\n";
  src += "#include \"lt_kernels_dev.h\"\n";
  // waves per SIMD the analyze kernel is built for (LT_JIT_WAVES, A/B runs; 4: <= 128 VGPRs)
  const char* we = getenv("LT_JIT_WAVES");
  const int waves = we && atoi(we) >= 1 && atoi(we) <= 8 ? atoi(we) : 4;
  char k[1024];
  // phase cuts (timing-only A/B runs, wrong outputs): LT_JIT_DEFINES=LT_JIT_STOP_AFTER=k ends
  // every pixel after phase k of lt_fast.h (0 winner pick, 1 despike, 2 DP, 3 fits + output)
  src += "#ifdef LT_JIT_STOP_AFTER\nstruct lt_jit_probe { static constexpr int kStopAfter = "
         "LT_JIT_STOP_AFTER; __device__ void mark(int) const {} };\n#else\n"
         "using lt_jit_probe = lt::NoProbe;\n#endif\n";
  snprintf(k, sizeof k,
           "extern \"C\" __global__ __launch_bounds__(64, %d) void lt_jit_analyze(const "
           "lt::KernelArgs A) {\n  (void)A;\n  lt::analyze_body<%d, %d, %s, lt_jit_probe>();\n}\n"
           "extern \"C\" __global__ __launch_bounds__(64, 4) void lt_jit_resolve(const "
           "lt::KernelArgs A) {\n  (void)A;\n  lt::resolve_body<%d, %d, %s>();\n}\n",
           waves, maxy, rmax, vt, maxy, rmax, vt);
  src += k;
  // the values binary32 cannot hold: a binary64 resolve (a binary64 series uses lt_jit_resolve
  // for both lists, as the product launches its one instance twice; an int16 series has none)
  if (strcmp(vt, "float") == 0) {
    snprintf(k, sizeof k,
             "extern \"C\" __global__ __launch_bounds__(64, 4) void lt_jit_resolve64(const "
             "lt::KernelArgs A) {\n  (void)A;\n  lt::resolve_body<%d, %d, double>();\n}\n",
             maxy, rmax);
    src += k;
  }
  return src;
}

// compile (or load from the disk cache) and load the module; false with err set
inline bool build(const std::string& src, const std::string& arch, int device,
                  lt_jit_kernels& out, std::string& err) {
  const std::string dir = src_dir();
  const std::string arch_opt = "--offload-arch=" + arch;  // the device's full target id
  const std::string inc_opt = "-I" + dir;
  std::vector<const char*> opts = {arch_opt.c_str(), "-O3", "-ffp-contract=off", "-std=c++17",
                                   inc_opt.c_str()};
  // cache key: the source, the options and every kernel header the source includes
  uint64_t h = fnv1a(src);
  for (const char* o : opts) h = fnv1a(o, h);
  for (const char* f : {"lt_kernels_dev.h", "lt_fast.h", "lt_pixel.h", "lt_lapack.h"}) {
    std::string text;
    if (!read_file(dir + "/" + f, text)) {
      err = "JIT: kernel header " + dir + "/" + f + " not found (LT_SRC_DIR)";
      return false;
    }
    h = fnv1a(text, h);
  }
  {
    std::string text;
    if (read_file(dir + "/../../include/lt_abi.h", text)) h = fnv1a(text, h);
  }
  const std::string cdir = cache_dir(dir);
  char name[64];
  snprintf(name, sizeof name, "/lt_jit_%016llx.co", (unsigned long long)h);
  const std::string cpath = cdir.empty() ? "" : cdir + name;
  std::string code;
  if (cpath.empty() || !read_file(cpath, code) || code.empty()) {
    hiprtcProgram rp;
    if (hiprtcCreateProgram(&rp, src.c_str(), "lt_jit.hip", 0, nullptr, nullptr) !=
        HIPRTC_SUCCESS) {
      err = "hiprtcCreateProgram failed";
      return false;
    }
    const hiprtcResult rc = hiprtcCompileProgram(rp, (int)opts.size(), opts.data());
    if (rc != HIPRTC_SUCCESS) {
      size_t n = 0;
      hiprtcGetProgramLogSize(rp, &n);
      std::string log(n, '\0');
      if (n) hiprtcGetProgramLog(rp, &log[0]);
      hiprtcDestroyProgram(&rp);
      err = "hiprtc (JIT analyze kernel): " + log.substr(0, 2000);
      return false;
    }
    size_t code_size = 0;
    hiprtcGetCodeSize(rp, &code_size);
    code.assign(code_size, '\0');
    hiprtcGetCode(rp, &code[0]);
    hiprtcDestroyProgram(&rp);
    if (!cpath.empty()) {  // best effort: a cache that cannot be written is skipped
      for (size_t i = 1; i <= cdir.size(); i++)  // mkdir -p
        if (i == cdir.size() || cdir[i] == '/') mkdir(cdir.substr(0, i).c_str(), 0755);
      const std::string tmp = cpath + "." + std::to_string((long long)getpid());
      FILE* f = fopen(tmp.c_str(), "wb");
      if (f) {
        const bool ok = fwrite(code.data(), 1, code.size(), f) == code.size();
        fclose(f);
        if (!ok || rename(tmp.c_str(), cpath.c_str()) != 0) remove(tmp.c_str());
      }
    }
  }
  if (hipModuleLoadData(&out.mod, code.data()) != hipSuccess ||
      hipModuleGetFunction(&out.analyze, out.mod, "lt_jit_analyze") != hipSuccess ||
      hipModuleGetFunction(&out.resolve, out.mod, "lt_jit_resolve") != hipSuccess) {
    if (out.mod) (void)hipModuleUnload(out.mod);
    out = lt_jit_kernels{};
    err = "JIT module load failed";
    return false;
  }
  // (a binary64 resolve exists for the non-int16 series types only: a failed lookup would leave
  // "named symbol not found" as HIP's last error for the next launch check to find)
  if (src.find("lt_jit_resolve64") != std::string::npos &&
      hipModuleGetFunction(&out.resolve64, out.mod, "lt_jit_resolve64") != hipSuccess) {
    (void)hipModuleUnload(out.mod);
    out = lt_jit_kernels{};
    err = "JIT module load failed (lt_jit_resolve64)";
    return false;
  }
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      cus < 1)
    cus = 256;
  auto grid = [&](hipFunction_t f) {
    int per_cu = 0;
    if (!f || hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, 64, 0) !=
                  hipSuccess || per_cu < 1)
      per_cu = 1;
    return (unsigned)(per_cu * cus);
  };
  out.resolve_grid = grid(out.resolve);
  out.resolve64_grid = grid(out.resolve64);
  return true;
}

}  // namespace lt_jit
