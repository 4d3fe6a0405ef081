/*
 * lt_abi.h — C ABI of the MI355X LandTrendr analysis engine (land_trendr_amd/liblt_hip.so).
 *
 * Drop-in boundary for the reference's per-pixel hot path. The reference is pure Python and binds
 * no native code; this ABI replaces, per batched tile of pixels:
 *   - utils.analyze(pix_datas, line_cost, target_date)        /root/reference/utils.py:735-789
 *       pick_winners :491-521, dicts2timeseries :523-532, despike :556-582,
 *       timeseries2int_series :534-554, least_squares :584-598, segmented_least_squares :600-631,
 *       find_segments :633-644, vertices2eqns :646-669, eqns2fitted_points :682-722
 *   - utils.change_labeling(trendline, label_rules)          /root/reference/utils.py:795-820
 *       Trendline.parse_disturbances / match_rule             /root/reference/classes.py:156-232
 *   - the per-pixel loop of MRLandTrendrJob.analysis_reducer  /root/reference/mr_land_trendr_job.py:83-126
 *     (one call per grid point there; one call per pixel tile here).
 * The Python host (land_trendr_amd/utils.py, classes.py) binds it with ctypes; INTEGRATION.md shows
 * the binding. Plain C types only: no torch types cross this boundary.
 *
 * Memory: the caller owns every buffer. lt_tile_in / lt_tile_out pointers are DEVICE pointers
 * (hipMalloc or torch tensors on the context's device); lt_scene / lt_params are HOST structs that
 * the call copies. Any lt_tile_out pointer may be NULL: that field is not written.
 * Layout: pixel-major structure of arrays. Plane q of a field starts at base + q*stride, the pixel
 * index runs fastest, so lane i of a wavefront touches element i of a plane (coalesced).
 */
#ifndef LT_ABI_H
#define LT_ABI_H
#ifndef __HIPCC_RTC__  /* hiprtc (the JIT kernels) brings its own */
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define LT_ABI_VERSION 7
#define LT_MAX_YEARS 64   /* distinct calendar years per scene (T <= 40 in every config) */
#define LT_MAX_OBS 1024   /* observations per scene (K*T) */
#define LT_MAX_RULES 16
#define LT_NODATA (-99)   /* settings.py:16 */
#define LT_MAX_TILE_PIX (1LL << 28) /* pixels per analyzed tile (lt_tile_in.n_pix)           */

/* Per-pixel status bits (lt_tile_out.status). Non-zero = the reference raises for this pixel. */
enum {
  LT_ST_OK = 0,
  LT_ST_EMPTY = 1,              /* no valid observation: reference IndexError (utils.py:569)     */
  LT_ST_SINGLE_YEAR = 2,        /* T == 1: reference ValueError in despike (utils.py:582)        */
  LT_ST_PRE_THRESHOLD_ATTR = 4, /* pre_threshold in reference mode: AttributeError (classes.py:207) */
  LT_ST_FEB29 = 8,              /* Feb-29 target in a non-leap year: ValueError (utils.py:511)   */
  LT_ST_NUMERIC = 16            /* LAPACK path not emulated (rank < 2 / DLASCL rescaling)        */
};

/* Return codes of the API functions. */
enum {
  LT_OK = 0,
  LT_ERR_ARG = -1,
  LT_ERR_HIP = -2,
  LT_ERR_JIT = -3,
  LT_ERR_LIMIT = -4
};

enum { LT_CT_NONE = 0, LT_CT_FD = 1, LT_CT_GD = 2, LT_CT_LD = 3 };          /* classes.py:44-47 */
enum { LT_Q_UNSET = 0, LT_Q_EQ = 1, LT_Q_LE = 2, LT_Q_GE = 3, LT_Q_GT = 4, LT_Q_LT = 5,
       LT_Q_OTHER = 9 /* set, but a qualifier match_rule ignores (classes.py:190-211) */ };
enum { LT_PRE_REFERENCE = 0, LT_PRE_DOCUMENTED = 1 };                      /* SURVEY App. B #1 */

/* One validated LabelRule (classes.py:32-64). The host performs the validation. */
typedef struct {
  int32_t change_type;   /* LT_CT_*                                  */
  int32_t onset_op;      /* LT_Q_UNSET / EQ / LE / GE / OTHER        */
  int32_t duration_op;   /* LT_Q_UNSET / GT / LT / OTHER             */
  int32_t pre_op;        /* LT_Q_UNSET / GT / LT / OTHER             */
  double onset_val;
  double duration_val;
  double pre_val;
  int32_t class_val;     /* rule.val, written to the class raster    */
  int32_t _pad;
} lt_rule;

/* settings.json semantics (README.md:46-85) minus target_date, which is folded into lt_scene. */
typedef struct {
  double line_cost;
  int32_t n_rules;
  int32_t pre_threshold_mode; /* LT_PRE_* */
  lt_rule rules[LT_MAX_RULES];
} lt_params;

/* Observation metadata shared by every pixel of a tile (all pixels of a co-registered stack see
 * the same acquisition dates). Built on the host from the dates and target_date
 * (land_trendr_amd/scene.py restates pick_winners' grouping, utils.py:503-517). */
typedef struct {
  int32_t n_obs;              /* K                                                          */
  int32_t n_years;            /* Y distinct calendar years, ascending                       */
  const int32_t* year;        /* [Y]   calendar year of slot y                              */
  const int32_t* slot_begin;  /* [Y+1] slot y covers order[slot_begin[y] .. slot_begin[y+1]) */
  const int32_t* order;       /* [K]   obs ids grouped by slot, caller's input order inside  */
  const int32_t* dist;        /* [K]   abs((target(year) - date).days) for order[k]          */
  const uint8_t* feb29_bad;   /* [Y]   1: target is Feb-29 and year y is not a leap year     */
} lt_scene;

/* Element types of raster planes (the GDAL band types a LandTrendr stack meets). */
enum { LT_T_F64 = 0, LT_T_I16 = 1, LT_T_U16 = 2, LT_T_I32 = 3, LT_T_F32 = 4, LT_T_U8 = 5,
       LT_T_U32 = 6, LT_T_I8 = 7, LT_T_I64 = 8 };
/* An index_eqn program that is an integer linear form (lt_index_linearize): every arithmetic
 * node has the one integer type wrap_type, multiplications have a constant side, no division.
 * Its value for bands b[0..n_bands) is store_out(wrap(c0 + sum coef[s] * b[s])), the sum taken
 * modulo 2^64 (exact modulo 2^bits(wrap_type), as numpy's wrapping node by node), store_out the
 * load stage's store into out_type (lt_index.h). The analyze kernel evaluates it on the winning
 * observations' band values, so the index raster is never written (lt_tile_in.obs_bands). */
#define LT_LIN_MAX_BANDS 4
typedef struct {
  int32_t n_bands;            /* band planes the form reads (<= LT_LIN_MAX_BANDS)            */
  int32_t band_type;          /* LT_T_* of the band planes (I16 / U16 / U8 / I32)            */
  int32_t wrap_type;          /* LT_T_* of every arithmetic node                             */
  int32_t out_type;           /* LT_T_* of the index raster the form stands for              */
  int64_t c0;                 /* constant term, modulo 2^64                                  */
  int64_t coef[LT_LIN_MAX_BANDS]; /* coefficient of band plane s, modulo 2^64                */
} lt_index_lin;

typedef struct lt_index lt_index;  /* a compiled index_eqn program (lt_index_compile) */

typedef struct {
  int64_t n_pix;              /* P                                                          */
  int64_t stride;             /* elements between obs planes (>= n_pix)                     */
  const double* obs_val;      /* [K][stride] observation values (float(val), utils.py:357)  */
  const uint8_t* obs_valid;   /* [K][stride] 0 = cloud-masked (utils.py:353); NULL = all    */
  const void* obs_index;      /* [K][stride] the index raster in its stored type (typically */
                              /* what lt_index_apply wrote); used instead of obs_val if set */
  int32_t index_type;         /* LT_T_* of obs_index                                       */
  int32_t _pad;
  /* fused load stage: when obs_bands is set, obs_val / obs_index are ignored and the value of
   * obs o at pixel p is lin evaluated on band s = obs_bands[o*band_obs_stride + s*band_stride +
   * p*band_pix_stride] (rast_algebra + its store, utils.py:447-484, per winner). Planar bands
   * (lt_index_io's layout): band_pix_stride 1, band_stride >= n_pix. Pixel-interleaved bands
   * (one pixel's n_bands values side by side): band_stride 1, band_pix_stride = n_bands — the
   * two int16 bands of 'B1 - B2' are then one 32-bit load per winner */
  const void* obs_bands;
  int64_t band_obs_stride;    /* elements between the bands of consecutive obs              */
  int64_t band_stride;        /* elements between bands of one obs at one pixel             */
  int64_t band_pix_stride;    /* elements between consecutive pixels of one band            */
  lt_index_lin lin;
  /* the cloud mask as bit planes: bit (o % 32) of obs_valid_bits[(o / 32)*stride + p] is 1 when
   * obs o is valid at pixel p (utils.py:353); used instead of obs_valid when set. The winner pick
   * then reads ceil(K/32) words per pixel instead of one byte per observation */
  const uint32_t* obs_valid_bits;
  /* fused load stage for ANY index_eqn program (ABI 6): with obs_bands set and index a program
   * from lt_index_compile, the value of obs o at pixel p is that program evaluated on the bands
   * above and stored into its out_type, as lt_index_apply writes it; lin is ignored. The analyze
   * and resolve kernels are then JIT-compiled (hiprtc) with the program inlined into the winner
   * pick, once per program and kernel instance (cached in the context and on disk, lt_jit.h). The
   * band planes have the program's band_type and n_bands; any band type, planar or interleaved */
  const lt_index* index;
} lt_tile_in;

/* ---- load stage: settings.json index_eqn (utils.py:447-484 rast_algebra) -------------------- */
#define LT_MAX_PROG 64
#define LT_MAX_BANDS 16
enum { LT_OP_BAND = 1,      /* push band plane ival (0-based slot), in band_type               */
       LT_OP_CONST_I = 2,   /* push the integer ival                                            */
       LT_OP_CONST_F = 3,   /* push the double fval                                             */
       LT_OP_ADD = 4, LT_OP_SUB = 5, LT_OP_MUL = 6,
       LT_OP_DIV = 7,       /* Python 2 '/': floor division on integer types, true on floats    */
       LT_OP_FLOORDIV = 8,  /* '//'                                                             */
       LT_OP_NEG = 9 };
/* One postfix operation. `type` is the numpy result type of the node (binary ops: both operands
 * are cast to it first, as numpy does); integer results wrap. */
typedef struct {
  int32_t op;
  int32_t type;               /* LT_T_*                                                     */
  int64_t ival;
  double fval;
} lt_index_op;
/* A typed program built and validated by the host (land_trendr_amd/index_eqn.py). */
typedef struct {
  int32_t n_ops;
  int32_t n_bands;            /* band planes per observation                                */
  int32_t band_type;          /* LT_T_* of every band plane                                 */
  int32_t out_type;           /* LT_T_* the index raster is stored in (the template's type) */
  lt_index_op ops[LT_MAX_PROG];
} lt_index_prog;
/* Device buffers of one lt_index_apply: band s of obs o, pixel p at
 * bands[o*obs_stride + s*band_stride + p*band_pix_stride]; index of obs o, pixel p at
 * out[o*out_stride + p]. Planar bands: band_pix_stride 1 (or 0), band_stride >= n_pix.
 * Pixel-interleaved bands (the layout lt_tile_in.obs_bands reads fastest): band_stride 1,
 * band_pix_stride = the program's n_bands. */
typedef struct {
  int64_t n_pix;
  int64_t n_obs;
  int64_t obs_stride;
  int64_t band_stride;
  int64_t out_stride;
  const void* bands;
  void* out;
  int64_t band_pix_stride;
} lt_index_io;

/* ---- settings.json compiled on the host (for non-Python hosts) -------------------------------- */
/* The Python exception the reference raises for a rejected settings.json (lt_settings_compile). */
enum { LT_EXC_NONE = 0, LT_EXC_VALUE = 1, LT_EXC_KEY = 2, LT_EXC_TYPE = 3, LT_EXC_ATTRIBUTE = 4,
       LT_EXC_ZERO_DIVISION = 5, LT_EXC_OTHER = 6 };
typedef struct {
  lt_params params;           /* line_cost + label_rules, validated as LabelRule does            */
  int32_t target_year;        /* target_date 'YYYY-MM-DD' (parse_date, utils.py:194-202)         */
  int32_t target_month;
  int32_t target_day;
  int32_t n_index_bands;      /* band numbers index_eqn reads, ascending (utils.py:219-225);    */
  int32_t index_bands[LT_MAX_BANDS]; /* band plane s of lt_index_io holds band index_bands[s]   */
  lt_index_prog index;        /* index_eqn as a typed program (n_ops = 0 if the key is absent)  */
} lt_settings;

typedef struct {
  int64_t stride;             /* elements between year / rule planes (>= n_pix)             */
  int32_t* status;            /* [P]    LT_ST_* bits                                        */
  int32_t* n_years;           /* [P]    T: years present for the pixel                      */
  int16_t* winner;            /* [Y][stride] winning obs id, -1 = year absent for the pixel */
  double* val_raw;            /* [Y][stride] TrendlinePoint fields (classes.py:67-116);     */
  double* val_fit;            /*             absent years are written NaN / 0               */
  double* fit_m;
  double* fit_b;
  double* right_m;
  double* right_b;
  uint8_t* spike;
  uint8_t* vertex;
  uint8_t* matched;           /* [R][stride] change_labeling (utils.py:795-820)             */
  int32_t* class_val;         /*             rule.val if matched else LT_NODATA             */
  int32_t* onset_year;        /*             LT_NODATA if unmatched                         */
  int32_t* duration;
  double* magnitude;          /*             LT_NODATA if unmatched                         */
  double* initial_val;
} lt_tile_out;

/* Input of the label stage alone: an already analysed trendline per pixel. */
typedef struct {
  int64_t n_pix;
  int64_t stride;             /* elements between year planes                               */
  int32_t n_years;            /* Y slots                                                    */
  const int32_t* year;        /* [Y] HOST array: calendar year of each slot                 */
  const double* val_fit;      /* [Y][stride] device                                         */
  const uint8_t* vertex;      /* [Y][stride] device                                         */
  const uint8_t* present;     /* [Y][stride] device, 0 = no point in this slot; NULL = all  */
} lt_label_in;

/* ---- output raster assembly (output_reducer -> data2raster, utils.py:414-440) ----------------- */
enum { LT_RASTER_REFERENCE = 0, /* the reference's file: holder cast, then GDT_Byte (App. B #5)   */
       LT_RASTER_TYPED = 1 };   /* the corrected file: each value in out_type, fill elsewhere      */
enum { LT_SEL_ALL = 0, LT_SEL_NONZERO = 1, LT_SEL_EQUALS = 2 };
/* One output key's raster from a plane in device memory. A grid point p contributes when the
 * selector holds (the reducer emitted the key for it: matched[r][p] != 0 for '<rule>_<field>',
 * winner[y][p] == obs id for 'trendline/<date>-<attr>'); raster pixel dest[p] then holds its value
 * (the reference's holder[y_off, x_off] = float(value)), every other pixel NODATA. */
typedef struct {
  int64_t n_pix;              /* grid points                                                 */
  const void* plane;          /* [n_pix] device values, or NULL: const_value for every point */
  int32_t plane_type;         /* LT_T_I32 / LT_T_F64 / LT_T_U8 / LT_T_I16                     */
  int32_t sel_kind;           /* LT_SEL_*                                                    */
  const void* sel;            /* [n_pix] device: uint8 (NONZERO) or int16 (EQUALS) plane      */
  int32_t sel_value;          /* EQUALS: the obs id                                          */
  int32_t holder_type;        /* REFERENCE: LT_T_* of the holder (template type promoted)    */
  double const_value;         /* plane == NULL: the value (class_val: rule.val)              */
  const int64_t* dest;        /* [n_pix] device raster offsets, all distinct; NULL: dest[p]=p */
  int64_t n_out;              /* raster pixels (rows * cols)                                 */
  int32_t mode;               /* LT_RASTER_*                                                 */
  int32_t out_type;           /* REFERENCE: LT_T_U8; TYPED: LT_T_I32 / LT_T_F64 / LT_T_U8     */
  double fill;                /* TYPED: value of the pixels no selected point reaches        */
  void* out;                  /* [n_out] device                                              */
} lt_raster_job;

typedef struct lt_ctx lt_ctx;

int lt_abi_version(void);

/* settings.json (README.md:46-85, read by get_settings utils.py:241 and analysis_reducer
 * mr_land_trendr_job.py:98-118) -> lt_settings, on the host, no context needed. Validates
 * label_rules exactly as LabelRule (classes.py:32-64) and parses target_date / index_eqn as the
 * Python host does (land_trendr_amd/classes.py, scene.py, index_eqn.py): band_type / out_type are
 * the LT_T_* of the analysis rasters and of the stored index (-1: band_type), raster_count the
 * rasters' band count (0: unchecked). On failure returns LT_ERR_ARG (LT_ERR_LIMIT: too many
 * rules), sets *exc_kind to the LT_EXC_* of the exception the reference raises and writes its
 * message into err (NUL-terminated, at most err_cap bytes). Replaces, for a native host, the
 * Python LabelRule / parse_date / index_eqn.IndexProgram steps. */
int lt_settings_compile(const char* settings_json, int32_t pre_threshold_mode, int32_t band_type,
                        int32_t out_type, int32_t raster_count, lt_settings* out,
                        int32_t* exc_kind, char* err, int64_t err_cap);
/* Bind a context to a HIP device. Not thread-safe: one context per thread / GPU. */
int lt_ctx_create(int device, lt_ctx** out);
int lt_ctx_destroy(lt_ctx* ctx);
const char* lt_last_error(const lt_ctx* ctx);

/* Full analyze + label of one tile, asynchronous on `stream` (a hipStream_t; NULL = default).
 * Kernels: (1) analyze — winner pick, despike, the lazy segmented-least-squares DP, fits and
 * labels for every pixel whose optimal path is decided without LAPACK emulation; (2) resolve —
 * the pixels (1) deferred, with the exact-OPT screened DP. Calls on one context are ordered by
 * the stream: do not use one context from two streams at once. */
int lt_analyze_tile(lt_ctx* ctx, const lt_scene* scene, const lt_params* params,
                    const lt_tile_in* in, const lt_tile_out* out, void* stream);

/* lt_analyze_tile over n_tiles tiles of one scene (the reducer loop over a batch of grid-point
 * tiles, mr_land_trendr_job.py:83-126). Tile t's resolve kernels run on the context's own side
 * stream beside tile t+1's analyze kernel; every output is complete in `stream` order once the
 * call's work is done (`stream` waits for the last resolve). Same results as n_tiles calls of
 * lt_analyze_tile. */
int lt_analyze_tiles(lt_ctx* ctx, const lt_scene* scene, const lt_params* params, int n_tiles,
                     const lt_tile_in* ins, const lt_tile_out* outs, void* stream);

/* lt_analyze_tiles where tile t's analyze kernel first waits on ready[t] (a recorded hipEvent_t,
 * or NULL = no wait; `ready` itself may be NULL). The load stage (parse_mapper's rast_algebra,
 * utils.py:447-484) of later tiles can then run on another stream beside this call's analyze
 * kernels instead of all of it ahead of the call. */
int lt_analyze_tiles_after(lt_ctx* ctx, const lt_scene* scene, const lt_params* params,
                           int n_tiles, const lt_tile_in* ins, const lt_tile_out* outs,
                           void* const* ready, void* stream);

/* lt_analyze_tiles_after that also records, for every tile t with done[t] != NULL, the caller's
 * hipEvent_t done[t] once every output of tile t is complete (`done` itself may be NULL), and
 * with join == 0 returns WITHOUT making `stream` wait for the tiles' last stages: the caller then
 * orders later work on the done events (ABI 7; a multi-GPU runner posts tile t's label send after
 * done[t], so tile t's resolve stage keeps running beside tile t+1's analyze kernel). */
int lt_analyze_tiles_ev(lt_ctx* ctx, const lt_scene* scene, const lt_params* params, int n_tiles,
                        const lt_tile_in* ins, const lt_tile_out* outs, void* const* ready,
                        void* const* done, int32_t join, void* stream);

/* change_labeling alone (utils.py:795-820) on trendlines already in device memory. Writes the
 * rule planes of `out` and out->status (only LT_ST_PRE_THRESHOLD_ATTR can be set). */
int lt_label_tile(lt_ctx* ctx, const lt_label_in* in, const lt_params* params,
                  const lt_tile_out* out, void* stream);

/* Output raster assembly: n_jobs rasters (lt_raster_job), asynchronous on `stream`: a fill of
 * every raster pixel with NODATA's converted value, then the selected grid points scattered in
 * (one pass when dest is NULL). Replaces data2raster's per-point loop (utils.py:429-438) and the
 * holder -> GDT_Byte conversion GDAL does in array2raster (utils.py:374-412). */
int lt_raster_assemble(lt_ctx* ctx, const lt_raster_job* jobs, int n_jobs, void* stream);
/* Which observations won some pixel's year (the acquisition dates that get trendline keys,
 * classes.py:100-116): bit o of bits[] (device, (n_obs + 31) / 32 words, zeroed by the call) is
 * set iff winner[y * stride + p] == o for some y < n_years, p < n_pix. Asynchronous on `stream`. */
int lt_winner_presence(lt_ctx* ctx, const int16_t* winner, int64_t stride, int32_t n_years,
                       int64_t n_pix, int32_t n_obs, uint32_t* bits, void* stream);

/* Stage timing: when enabled, each lt_analyze_tile brackets its kernels with hipEvents on the
 * launch stream; lt_ctx_stage_ms returns the accumulated milliseconds per stage
 * (0 = analyze: every pixel with the lazy DP, 1 = resolve: the deferred pixels with the exact-OPT
 * DP) since the last call, and the number of lt_analyze_tile calls. */
int lt_ctx_set_timing(lt_ctx* ctx, int enable);
int lt_ctx_stage_ms(lt_ctx* ctx, double* ms_out, int n_stages, int64_t* n_launches);
/* Pixels the last lt_analyze_tile deferred to the resolve stage (synchronous read). */
int lt_ctx_last_deferred(lt_ctx* ctx, int64_t* n_deferred);

/* Load stage. lt_index_codegen writes the HIP source generated for `prog` (for inspection and the
 * CPU tests; returns the length, or a negative LT_ERR_*). lt_index_compile builds it with hiprtc
 * for the context's device (cached per program inside the context; LT_ERR_JIT with the compiler
 * log in lt_last_error on failure). lt_index_apply computes the index raster of every observation
 * of a tile — rast_algebra's eval, then the store into out_type — asynchronously on `stream`. */
int lt_index_codegen(const lt_index_prog* prog, char* buf, int64_t cap);
int lt_index_compile(lt_ctx* ctx, const lt_index_prog* prog, lt_index** out);
int lt_index_apply(lt_ctx* ctx, const lt_index* fn, const lt_index_io* io, void* stream);
/* The linear form of `prog` (see lt_index_lin) for the analyze kernel's fused load stage, or
 * LT_ERR_ARG when the program is not one (a division, a float node, a product of two band
 * terms, mixed integer node types, a band type the kernel does not read, more than
 * LT_LIN_MAX_BANDS bands): such programs keep lt_index_apply. Host only, no context. */
int lt_index_linearize(const lt_index_prog* prog, lt_index_lin* out);

/* ---- JIT kernels (lt_tile_in.index; ABI 7) -------------------------------------------------------
 * A tile carrying an index_eqn program runs analyze / resolve kernels compiled for it (hiprtc,
 * lt_jit.h) from kernel headers embedded in this library. Until a tile's module is ready, or if its
 * compile fails, the tile runs on the precompiled kernels instead — a linear program through its
 * lt_index_lin form, any other through its index raster (the program's load kernel into a context
 * scratch buffer) — with the same results; lt_ctx_jit_stats counts both kinds of tile. */
enum { LT_JIT_SYNC = 0,    /* a launch needing a module compiles it first (the default)        */
       LT_JIT_ASYNC = 1 }; /* modules compile on worker threads; tiles launched before theirs
                              is ready take the precompiled kernels                             */
int lt_ctx_set_jit_mode(lt_ctx* ctx, int32_t mode);
/* Compile (wait != 0) or start compiling (wait == 0, on a worker thread) the module a
 * lt_analyze_tiles call with this scene, params, tile and output set would use, so that no launch
 * waits for hiprtc (e.g. every scene of a mosaic before the first tile). LT_OK also when `in`
 * carries no program; LT_ERR_JIT (the log in lt_last_error) when a waited-for compile failed. */
int lt_jit_prepare(lt_ctx* ctx, const lt_scene* scene, const lt_params* params,
                   const lt_tile_in* in, const lt_tile_out* out, int32_t wait);
typedef struct {
  int64_t jit_tiles;       /* tiles launched on JIT kernels                                    */
  int64_t fallback_tiles;  /* tiles with a program launched on the precompiled kernels         */
  int64_t compiles;        /* modules compiled with hiprtc                                     */
  int64_t disk_hits;       /* modules read from the disk cache (LT_JIT_CACHE)                  */
  int64_t failures;        /* modules whose compile or load failed                             */
  int64_t modules;         /* modules loaded now (least recently used unloaded past a cap)     */
  int64_t evictions;       /* modules unloaded                                                 */
  int64_t pending;         /* compiles still running                                           */
} lt_jit_stats;
/* The context's JIT counters since creation and the last JIT failure message (NUL-terminated into
 * last_error, at most cap bytes; may be NULL). Loads modules whose compile has finished. */
int lt_ctx_jit_stats(lt_ctx* ctx, lt_jit_stats* out, char* last_error, int64_t cap);
/* The module source the context would compile for a tile of this scene and params carrying
 * `prog` (masked: the tile has a cloud mask; year_out: a per-year plane is requested), with the
 * launch constants (LT_JIT_SRC_SPEC) and the scene's tables (LT_JIT_SRC_SCENE); host only, for
 * inspection and ahead-of-time builds. Returns the length, or a negative LT_ERR_*. */
enum { LT_JIT_SRC_SPEC = 1, LT_JIT_SRC_SCENE = 2, LT_JIT_SRC_FIELDS = 4 };
/* LT_JIT_SRC_FIELDS: flags bits 8.. carry the launch's non-null output planes as the kernels'
 * LT_FIELD_* bits (status 0, n_years 1, matched 2, class_val 3, onset_year 4, duration 5,
 * magnitude 6, initial_val 7, winner 8, val_raw 9, val_fit 10, fit_m 11, fit_b 12, right_m 13,
 * right_b 14, spike 15, vertex 16), as the context specialises a launch for them. */
int lt_jit_source(const lt_scene* scene, const lt_params* params, const lt_index_prog* prog,
                  int32_t masked, int32_t year_out, int32_t flags, char* buf, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif
