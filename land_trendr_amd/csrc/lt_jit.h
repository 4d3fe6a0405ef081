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
// One module per specialisation (program, MAXY, RMAX, series type, the launch constants of Spec),
// compiled on first use (~10 s) or ahead of the launches (lt_jit_prepare), on the launching thread
// or a worker (lt_ctx_set_jit_mode), and cached in the context (keyed by spec_key, least recently
// used modules unloaded past a cap, lt_abi.hip); the code object is also cached on disk
// (LT_JIT_CACHE, default <library dir>/../build/jit, at most kDiskCacheMax files) under a hash of
// the generated source, the kernel headers (embedded in the library), the compile options, the
// device's target id and the hiprtc / HIP runtime versions, so later processes load it at once.
#pragma once
#include <dirent.h>
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <string>
#include <vector>

#include "lt_index.h"
#include "lt_pixel.h"

struct lt_jit_kernels {
  hipModule_t mod = nullptr;
  hipFunction_t analyze = nullptr, resolve = nullptr, resolve64 = nullptr;
  unsigned resolve_grid = 0, resolve64_grid = 0;  // resident waves of each resolve kernel
  int wpb = 1;  // waves per workgroup of the analyze kernel (LT_JIT_WPB)
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

// The kernel headers the JIT kernels are compiled from, passed to hiprtc in memory under their bare
// file names. By default the copies compiled into this library (build/gen/lt_jit_embed.inc,
// written by __graft_entry__.embed_headers at build time): the JIT kernels then see exactly the
// KernelArgs / lt_tile_in / lt_params layouts the library's host code was compiled with, and no
// csrc/ tree is needed at run time. LT_SRC_DIR=<dir> (development only: header edits without a
// rebuild) reads <dir>/lt_*.h and <dir>/../../include/lt_abi.h instead; a missing one is a JIT
// failure, which the launch answers with the precompiled kernels (lt_abi.hip jit_fallback).
#if __has_include("lt_jit_embed.inc")
#include "lt_jit_embed.inc"
#endif

constexpr int kNHeaders = 5;
constexpr const char* kHeaderName[kNHeaders] = {"lt_abi.h", "lt_lapack.h", "lt_pixel.h",
                                                "lt_fast.h", "lt_kernels_dev.h"};

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

inline uint64_t fnv1a_bytes(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
  const unsigned char* c = (const unsigned char*)p;
  for (size_t i = 0; i < n; i++) {
    h ^= c[i];
    h *= 1099511628211ull;
  }
  return h;
}
inline uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
  return fnv1a_bytes(s.data(), s.size(), h);
}

struct Headers {
  std::vector<std::string> text;  // kNHeaders texts, in kHeaderName order
  uint64_t hash = 0;
  bool embedded = false;
};

// the headers (embedded, or LT_SRC_DIR's); false with err when one is missing
inline bool headers(Headers& H, std::string& err) {
  H.text.assign(kNHeaders, std::string());
  const char* dir = getenv("LT_SRC_DIR");
  if (!(dir && *dir)) {
#ifdef LT_JIT_EMBEDDED
    static_assert(kLtJitNHdr == kNHeaders, "embedded header list");
    for (int i = 0; i < kNHeaders; i++) {
      if (strcmp(kLtJitHdrName[i], kHeaderName[i]) != 0) {
        err = "JIT: embedded header list out of order";
        return false;
      }
      H.text[i] = kLtJitHdrText[i];
    }
    H.embedded = true;
#else
    // a library built without the embedded copies (a profiling variant): csrc/ beside it
    Dl_info info;
    static std::string lib_dir;
    if (lib_dir.empty() && dladdr((void*)&headers, &info) && info.dli_fname) {
      std::string p = info.dli_fname;
      const size_t s = p.rfind('/');
      lib_dir = (s == std::string::npos ? std::string(".") : p.substr(0, s)) + "/csrc";
    }
    dir = lib_dir.c_str();
#endif
  }
  if (!H.embedded) {
    const std::string d = dir;
    for (int i = 0; i < kNHeaders; i++) {
      const std::string path =
          i == 0 ? d + "/../../include/lt_abi.h" : d + "/" + kHeaderName[i];
      if (!read_file(path, H.text[i])) {
        err = "JIT: kernel header " + path + " not found (LT_SRC_DIR)";
        return false;
      }
      // the one relative include, as the embedded copies have it
      const std::string rel = "#include \"../../include/lt_abi.h\"";
      for (size_t at; (at = H.text[i].find(rel)) != std::string::npos;)
        H.text[i].replace(at, rel.size(), "#include \"lt_abi.h\"");
    }
  }
  uint64_t h = fnv1a(std::string(H.embedded ? "embedded" : "disk"));
  for (const std::string& t : H.text) h = fnv1a(t, h);
  H.hash = h;
  return true;
}

// the disk cache of code objects: LT_JIT_CACHE ("" disables it), else build/jit beside the
// library's package directory
inline std::string cache_dir() {
  const char* e = getenv("LT_JIT_CACHE");
  if (e) return e;
  Dl_info info;
  if (dladdr((void*)&cache_dir, &info) && info.dli_fname) {
    std::string p = info.dli_fname;
    const size_t s = p.rfind('/');
    return (s == std::string::npos ? std::string(".") : p.substr(0, s)) + "/../build/jit";
  }
  return "build/jit";
}

// at most this many code objects stay in the disk cache (the oldest by mtime go first)
constexpr int kDiskCacheMax = 64;

inline void prune_disk_cache(const std::string& dir) {
  DIR* d = opendir(dir.c_str());
  if (!d) return;
  std::vector<std::pair<double, std::string>> files;
  while (dirent* e = readdir(d)) {
    const std::string n = e->d_name;
    if (n.compare(0, 7, "lt_jit_") != 0 || n.size() < 3 || n.substr(n.size() - 3) != ".co")
      continue;
    struct stat st;
    const std::string path = dir + "/" + n;
    if (stat(path.c_str(), &st) == 0)
      files.emplace_back((double)st.st_mtim.tv_sec + 1e-9 * st.st_mtim.tv_nsec, path);
  }
  closedir(d);
  if ((int)files.size() <= kDiskCacheMax) return;
  std::sort(files.begin(), files.end());
  for (size_t i = 0; i + kDiskCacheMax < files.size(); i++) remove(files[i].second.c_str());
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
  bool masked = false, year_out = false, tl_split = false;
  lt_params params{};
  const lt::DevScene* scene = nullptr;  // the scene's tables as constants (LT_SPEC_SCENE)
  bool fields_on = false;  // the output planes as constants (LT_SPEC_FIELDS, lt_pixel.h LT_OUTF)
  uint32_t fields = 0;
  // with fields_on: the cloud mask comes as bit planes (obs_valid_bits, <= 128 observations) —
  // LT_SPEC_VBITS 1 — or as bytes (0)
  bool vbits = false;
  // with fields_on: two 16-bit bands pixel-interleaved (band_stride 1, band_pix_stride 2), the
  // tile 4-byte aligned with an even obs stride: one 32-bit load per winner (LT_SPEC_BAND_PAIR)
  bool band_pair = false;
  // with fields_on: the tile is a whole number of the analyze kernel's workgroups (every lane of
  // every wave has a pixel: LT_SPEC_FULL)
  bool full = false;
};

// The planes a module is specialised as present: the launch's, plus winner / val_raw kept as
// run-time pointers for the multi-rule instances. With those two planes compile-time null the
// winner pick keeps only its branch-free store loop: c2 (one rule) 3082 vs 2848 Mpx/s, but the
// c3 instance (four rule slots) 2157 vs 2225 (same box, profiles/r06_run9, r06_run10)
inline uint32_t spec_fields(uint32_t launch_mask, int rmax) {
  return launch_mask | (rmax > 1 ? (LT_FIELD_winner | LT_FIELD_val_raw) : 0u);
}

// The launch's non-null output planes as LT_FIELD_* bits (lt_pixel.h)
inline uint32_t out_field_mask(const lt_tile_out* o) {
  uint32_t m = 0;
#define LT_JIT_FIELD(f) \
  if (o->f) m |= LT_FIELD_##f;
  LT_JIT_FIELD(status) LT_JIT_FIELD(n_years) LT_JIT_FIELD(matched) LT_JIT_FIELD(class_val)
  LT_JIT_FIELD(onset_year) LT_JIT_FIELD(duration) LT_JIT_FIELD(magnitude)
  LT_JIT_FIELD(initial_val) LT_JIT_FIELD(winner) LT_JIT_FIELD(val_raw) LT_JIT_FIELD(val_fit)
  LT_JIT_FIELD(fit_m) LT_JIT_FIELD(fit_b) LT_JIT_FIELD(right_m) LT_JIT_FIELD(right_b)
  LT_JIT_FIELD(spike) LT_JIT_FIELD(vertex)
#undef LT_JIT_FIELD
  return m;
}

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

// The environment switches that change the generated source (A/B runs: LT_JIT_DEFINES adds
// compile-time switches, LT_JIT_WAVES the analyze kernel's occupancy): part of spec_key
inline std::string env_switches() {
  std::string r;
  for (const char* v : {"LT_JIT_DEFINES", "LT_JIT_WAVES", "LT_JIT_WPB", "LT_JIT_OVERRIDE_DIR",
                        "LT_JIT_FIELDS", "LT_JIT_FIELDS_OR", "LT_JIT_FULL"}) {
    const char* e = getenv(v);
    r += std::string(v) + "=" + (e ? e : "") + ";";
  }
  return r;
}

// Waves per workgroup of the JIT analyze kernel (LT_JIT_WPB = 1, 2 or 4; default 1): each wave still
// analyses its own 64 pixels with its own LDS slice; a workgroup of several takes one contiguous
// run of 64 * wpb pixels, so its waves' pieces of each per-year row lie side by side
inline int analyze_wpb() {
  const char* e = getenv("LT_JIT_WPB");
  const int w = e ? atoi(e) : 1;
  return (w == 2 || w == 4) ? w : 1;
}

// The identity of the module source() generates for these inputs, without generating it: the
// context's module map is keyed on it (a tile launch hashes ~10 KB of scene tables instead of
// formatting and comparing the whole source)
inline uint64_t spec_key(const lt_index_prog& P, int maxy, int rmax, const char* vt,
                         const Spec& sp) {
  uint64_t h = fnv1a_bytes(&P.n_ops, sizeof P.n_ops);
  h = fnv1a_bytes(&P.n_bands, sizeof P.n_bands, h);
  h = fnv1a_bytes(&P.band_type, sizeof P.band_type, h);
  h = fnv1a_bytes(&P.out_type, sizeof P.out_type, h);
  for (int i = 0; i < P.n_ops && i < LT_MAX_PROG; i++) {
    const lt_index_op& o = P.ops[i];
    h = fnv1a_bytes(&o.op, sizeof o.op, h);
    h = fnv1a_bytes(&o.type, sizeof o.type, h);
    h = fnv1a_bytes(&o.ival, sizeof o.ival, h);
    h = fnv1a_bytes(&o.fval, sizeof o.fval, h);
  }
  const int inst[3] = {maxy, rmax, (int)strlen(vt)};
  h = fnv1a_bytes(inst, sizeof inst, fnv1a(std::string(vt), h));
  const int flags[8] = {sp.on ? 1 : 0, sp.n_years, sp.masked ? 1 : 0, sp.year_out ? 1 : 0,
                        sp.tl_split ? 1 : 0, sp.fields_on ? 1 : 0, (int)sp.fields,
                        (sp.vbits ? 1 : 0) | (sp.band_pair ? 2 : 0) | (sp.full ? 4 : 0)};
  h = fnv1a_bytes(flags, sizeof flags, h);
  if (sp.on) {
    const lt_params& Q = sp.params;
    h = fnv1a_bytes(&Q.line_cost, sizeof Q.line_cost, h);
    h = fnv1a_bytes(&Q.n_rules, sizeof Q.n_rules, h);
    h = fnv1a_bytes(&Q.pre_threshold_mode, sizeof Q.pre_threshold_mode, h);
    for (int r = 0; r < Q.n_rules && r < LT_MAX_RULES; r++) {
      const lt_rule& u = Q.rules[r];
      const int32_t ints[5] = {u.change_type, u.onset_op, u.duration_op, u.pre_op, u.class_val};
      const double dbl[3] = {u.onset_val, u.duration_val, u.pre_val};
      h = fnv1a_bytes(dbl, sizeof dbl, fnv1a_bytes(ints, sizeof ints, h));
    }
  }
  if (sp.on && sp.scene) {
    const lt::DevScene& S = *sp.scene;
    h = fnv1a_bytes(&S.n_obs, sizeof S.n_obs, h);
    h = fnv1a_bytes(&S.n_years, sizeof S.n_years, h);
    h = fnv1a_bytes(&S.feb29_mask, sizeof S.feb29_mask, h);
    const int Y = S.n_years, K = S.n_obs;
    h = fnv1a_bytes(S.year, sizeof(int32_t) * Y, h);
    h = fnv1a_bytes(S.slot_begin, sizeof(int32_t) * (Y + 1), h);
    h = fnv1a_bytes(S.order, sizeof(int32_t) * K, h);
    h = fnv1a_bytes(S.dist, sizeof(int32_t) * K, h);
    h = fnv1a_bytes(S.winner_all, sizeof(int32_t) * Y, h);
  } else {
    h = fnv1a(std::string("no-scene"), h);
  }
  return fnv1a(env_switches(), h);
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
             "#include \"lt_abi.h\"\n#define LT_SPEC_Y %d\n#define LT_SPEC_MASKED %d\n"
             "#define LT_SPEC_YEAR_OUT %d\n#define LT_SPEC_TL_SPLIT %d\n#define LT_SPEC_NRULES %d\n"
             "#define LT_SPEC_PRE_MODE %d\n#define LT_SPEC_LINE_COST %a\n",
             sp.n_years, sp.masked ? 1 : 0, sp.year_out ? 1 : 0, sp.tl_split ? 1 : 0, Q.n_rules,
             Q.pre_threshold_mode, Q.line_cost);
    src += d;
    if (sp.fields_on) {
      snprintf(d, sizeof d,
               "#define LT_SPEC_FIELDS 0x%xu\n#define LT_SPEC_VBITS %d\n#define LT_SPEC_BAND_PAIR %d\n"
               "#define LT_SPEC_FULL %d\n",
               (unsigned)sp.fields, sp.vbits ? 1 : 0, sp.band_pair ? 1 : 0, sp.full ? 1 : 0);
      src += d;
    }
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
  const int wpb = analyze_wpb();
  src += "#define LT_WPB " + std::to_string(wpb) + "\n";
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
           "extern \"C\" __global__ __launch_bounds__(%d, %d) void lt_jit_analyze(const "
           "lt::KernelArgs A) {\n  (void)A;\n  lt::analyze_body<%d, %d, %s, lt_jit_probe>();\n}\n"
           "extern \"C\" __global__ __launch_bounds__(64, 4) void lt_jit_resolve(const "
           "lt::KernelArgs A) {\n  (void)A;\n  lt::resolve_body<%d, %d, %s>();\n}\n",
           64 * wpb, waves, maxy, rmax, vt, maxy, rmax, vt);
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

// The identity of everything a module's code depends on besides its source: the kernel headers,
// the compile options, the hiprtc and HIP runtime versions (the device's target id is one of the
// options). The disk cache's file name is its hash with the source's.
inline uint64_t env_key(const Headers& H, const std::vector<std::string>& opts) {
  uint64_t h = H.hash;
  for (const std::string& o : opts) h = fnv1a(o, h);
  int maj = 0, min = 0, rt = 0;
  (void)hiprtcVersion(&maj, &min);
  (void)hipRuntimeGetVersion(&rt);
  const int v[3] = {maj, min, rt};
  return fnv1a_bytes(v, sizeof v, h);
}

inline std::vector<std::string> options(const std::string& arch) {
  return {"--offload-arch=" + arch, "-O3", "-ffp-contract=off", "-std=c++17"};
}

// Compile `src` for `arch` into a code object (or read it from the disk cache). Host work only —
// hiprtc and file IO, no HIP runtime call that touches the device — so it may run on a worker
// thread (lt_abi.hip LT_JIT_ASYNC). false with err set.
inline bool compile(const std::string& src, const std::string& arch, std::string& code,
                    bool& disk_hit, std::string& err) {
  disk_hit = false;
  // A/B runs of post-compile variants (tools/jit_asm.py): LT_JIT_OVERRIDE_DIR/lt_src_<FNV-1a of
  // the source>.co is loaded instead of compiling this source
  if (const char* od = getenv("LT_JIT_OVERRIDE_DIR")) {
    char nm[64];
    snprintf(nm, sizeof nm, "/lt_src_%016llx.co", (unsigned long long)fnv1a(src));
    if (read_file(std::string(od) + nm, code) && !code.empty()) {
      disk_hit = true;
      return true;
    }
  }
  Headers H;
  if (!headers(H, err)) return false;
  const std::vector<std::string> opts = options(arch);
  const uint64_t h = fnv1a(src, env_key(H, opts));
  const std::string cdir = cache_dir();
  char name[64];
  snprintf(name, sizeof name, "/lt_jit_%016llx.co", (unsigned long long)h);
  const std::string cpath = cdir.empty() ? "" : cdir + name;
  if (!cpath.empty() && read_file(cpath, code) && !code.empty()) {
    disk_hit = true;
    return true;
  }
  std::vector<const char*> hdr_text, hdr_name;
  for (int i = 0; i < kNHeaders; i++) {
    hdr_text.push_back(H.text[i].c_str());
    hdr_name.push_back(kHeaderName[i]);
  }
  hiprtcProgram rp;
  if (hiprtcCreateProgram(&rp, src.c_str(), "lt_jit.hip", kNHeaders, hdr_text.data(),
                          hdr_name.data()) != HIPRTC_SUCCESS) {
    err = "hiprtcCreateProgram failed";
    return false;
  }
  std::vector<const char*> o;
  for (const std::string& s : opts) o.push_back(s.c_str());
  const hiprtcResult rc = hiprtcCompileProgram(rp, (int)o.size(), o.data());
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
    const std::string tmp = cpath + "." + std::to_string((long long)getpid()) + "." +
                            std::to_string((unsigned long long)(uintptr_t)&code);
    FILE* f = fopen(tmp.c_str(), "wb");
    if (f) {
      const bool ok = fwrite(code.data(), 1, code.size(), f) == code.size();
      fclose(f);
      if (!ok || rename(tmp.c_str(), cpath.c_str()) != 0) remove(tmp.c_str());
    }
    prune_disk_cache(cdir);
  }
  return true;
}

// load a code object as a module on the calling thread's device; false with err set
inline bool load(const std::string& code, bool has_resolve64, int device, lt_jit_kernels& out,
                 std::string& err) {
  if (hipModuleLoadData(&out.mod, code.data()) != hipSuccess ||
      hipModuleGetFunction(&out.analyze, out.mod, "lt_jit_analyze") != hipSuccess ||
      hipModuleGetFunction(&out.resolve, out.mod, "lt_jit_resolve") != hipSuccess) {
    if (out.mod) (void)hipModuleUnload(out.mod);
    out = lt_jit_kernels{};
    (void)hipGetLastError();
    err = "JIT module load failed";
    return false;
  }
  // (a binary64 resolve exists for the non-int16 series types only: a failed lookup would leave
  // "named symbol not found" as HIP's last error for the next launch check to find)
  if (has_resolve64 &&
      hipModuleGetFunction(&out.resolve64, out.mod, "lt_jit_resolve64") != hipSuccess) {
    (void)hipModuleUnload(out.mod);
    out = lt_jit_kernels{};
    (void)hipGetLastError();
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
  out.wpb = analyze_wpb();  // as source() generated it (the same environment)
  return true;
}

}  // namespace lt_jit
