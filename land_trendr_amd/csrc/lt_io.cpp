// lt_io.cpp — host codecs of the raster IO around the hot path (include/lt_io.h): TIFF LZW
// (Compression = 5) decode and encode, the compression GDAL writes for the reference
// (array2raster's COMPRESS=LZW, utils.py:386) and reads back (ds2array, utils.py:272-282).
//
// The TIFF 6.0 LZW variant: codes packed most significant bit first, 9 to 12 bits wide,
// ClearCode 256, EndOfInformation 257, first free code 258, and the "early change" of libtiff
// (the width grows when the next free code reaches 2^width - 1, one code before it would stop
// fitting). The encoder follows libtiff's LZWEncode / LZWPostEncode: a Clear code first, a Clear
// when the table holds 4094 entries, and the width step taken before EndOfInformation.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/lt_io.h"

namespace {

constexpr int kClear = 256, kEoi = 257, kFirst = 258, kMaxBits = 12;

struct BitWriter {
  uint8_t* out;
  int64_t cap, n = 0;
  uint64_t acc = 0;  // the pending bits, the oldest most significant (codes <= 12 bits)
  int nacc = 0;
  bool overflow = false;
  void put(int code, int nbits) {
    acc = (acc << nbits) | (uint32_t)code;
    nacc += nbits;
    if (nacc >= 32) {  // four bytes at a time (MSB first)
      nacc -= 32;
      const uint32_t w = (uint32_t)(acc >> nacc);
      if (__builtin_expect(n + 4 <= cap, 1)) {
        const uint32_t be = __builtin_bswap32(w);
        memcpy(out + n, &be, 4);
        n += 4;
      } else {
        for (int k = 3; k >= 0; k--) byte((uint8_t)(w >> (8 * k)));
      }
      acc &= (1ull << nacc) - 1ull;
    }
  }
  void byte(uint8_t b) {
    if (n < cap) out[n] = b;
    else overflow = true;
    n++;
  }
  void flush() {
    while (nacc >= 8) {
      nacc -= 8;
      byte((uint8_t)(acc >> nacc));
    }
    if (nacc > 0) byte((uint8_t)(acc << (8 - nacc)));
    nacc = 0;
    acc = 0;
  }
};

}  // namespace

extern "C" {

int64_t lt_lzw_decode(const uint8_t* in, int64_t n_in, uint8_t* out, int64_t cap) {
  if (!in || n_in < 0 || (cap > 0 && !out)) return LT_IO_ERR_ARG;
  if (cap >= (int64_t)1 << 31) return LT_IO_ERR_ARG;  // strips are far smaller (32-bit positions)
  // Every string of the table is already in `out`: code c >= kFirst is the len[c] bytes at src[c]
  // (where it was last written), so emitting is a copy from earlier output and a new entry is
  // (the previous emission's start, its length + 1): no per-byte chain walk. A literal c is the
  // one byte at kLit + c, so literals and strings take one path. The table lives on the stack (a
  // thread_local one in a -fPIC library costs a __tls_get_addr call per access).
  static const struct LitBytes {
    uint8_t b[256 + 16];
    LitBytes() {
      for (int c = 0; c < 256; c++) b[c] = (uint8_t)c;
      for (int c = 256; c < 256 + 16; c++) b[c] = 0;  // the 16-byte copy's slack
    }
  } kLit;
  const uint8_t* src[4096];
  uint16_t len[4096];
  for (int c = 0; c < 256; c++) {
    src[c] = kLit.b + c;
    len[c] = 1;
  }
  int nbits = 9, free_ent = kFirst, grow_at = (1 << 9) - 1;
  uint32_t mask = (1u << 9) - 1u;
  int64_t n_out = 0;
  int64_t bitpos = 0;
  const int64_t nbits_in = n_in * 8;
  const int64_t fast_end = (n_in - 4) * 8;  // a 32-bit load at bitpos >> 3 stays inside `in`
  uint8_t* const out_end = out + cap;
  // the next code (MSB first): one unaligned big-endian 32-bit load while 4 bytes remain, else a
  // byte at a time; -1 when the input cannot fill a whole code (the strip's end)
  auto get = [&]() -> int {
    if (__builtin_expect(bitpos <= fast_end, 1)) {
      uint32_t w;
      memcpy(&w, in + (bitpos >> 3), 4);
      w = __builtin_bswap32(w);
      const int code = (int)((w >> (32 - nbits - (int)(bitpos & 7))) & mask);
      bitpos += nbits;
      return code;
    }
    if (bitpos + nbits > nbits_in) return -1;
    uint32_t acc = 0;
    for (int k = 0; k < nbits; k++, bitpos++)
      acc = (acc << 1) | ((in[bitpos >> 3] >> (7 - (bitpos & 7))) & 1u);
    return (int)acc;
  };
  // copy L bytes from s (earlier output or kLit, no overlap with what is written) to d
  auto copy = [&](uint8_t* d, const uint8_t* s, int L) {
    if (__builtin_expect(L <= 16 && d + 16 <= out_end, 1)) {  // two unaligned 8-byte moves
      uint64_t a, b;                                          // (the slack is output space
      memcpy(&a, s, 8);                                       // later codes overwrite)
      memcpy(&b, s + 8, 8);
      memcpy(d, &a, 8);
      if (L > 8) memcpy(d + 8, &b, 8);
    } else {
      for (int k = 0; k < L; k++) d[k] = s[k];
    }
  };
  uint32_t old_pos = 0;  // the previous code's emission
  int old_len = 0;
  bool have_old = false;
  for (;;) {
    int code = get();
    if (code < 0 || code == kEoi) break;  // a strip may end without EOI (libtiff tolerates it)
    if (code == kClear) {
      nbits = 9;
      mask = (1u << 9) - 1u;
      grow_at = (1 << 9) - 1;
      free_ent = kFirst;
      code = get();
      if (code < 0 || code == kEoi) break;
      if (code >= 256) return LT_IO_ERR_DATA;
      if (n_out >= cap) return LT_IO_ERR_SPACE;
      out[n_out] = (uint8_t)code;
      old_pos = (uint32_t)n_out++;
      old_len = 1;
      have_old = true;
      continue;
    }
    if (__builtin_expect(!have_old, 0)) {  // data must start with a Clear code or a literal
      if (code >= 256) return LT_IO_ERR_DATA;
      if (n_out >= cap) return LT_IO_ERR_SPACE;
      out[n_out] = (uint8_t)code;
      old_pos = (uint32_t)n_out++;
      old_len = 1;
      have_old = true;
      continue;
    }
    if (code < free_ent) {  // a literal or a table string
      const int L = len[code];
      if (n_out + L > cap) return LT_IO_ERR_SPACE;
      copy(out + n_out, src[code], L);
      if (free_ent < 4096) {  // previous string + this one's first byte: contiguous in out
        src[free_ent] = out + old_pos;
        len[free_ent] = (uint16_t)(old_len + 1);
        free_ent++;
      }
      old_pos = (uint32_t)n_out;
      old_len = L;
      n_out += L;
    } else if (code == free_ent && free_ent < 4096) {
      // KwKwK: the previous string + its own first byte
      const int L = old_len + 1;
      if (n_out + L > cap) return LT_IO_ERR_SPACE;
      uint8_t* d = out + n_out;
      const uint8_t* s = out + old_pos;
      copy(d, s, old_len);
      d[old_len] = s[0];
      src[free_ent] = d;
      len[free_ent] = (uint16_t)L;
      free_ent++;
      old_pos = (uint32_t)n_out;
      old_len = L;
      n_out += L;
    } else {
      return LT_IO_ERR_DATA;
    }
    if (free_ent >= grow_at && nbits < kMaxBits) {
      nbits++;
      mask = (1u << nbits) - 1u;
      grow_at = (1 << nbits) - 1;
    }
  }
  return n_out;
}

int64_t lt_lzw_encode(const uint8_t* in, int64_t n_in, uint8_t* out, int64_t cap) {
  if (!in || n_in < 0 || (cap > 0 && !out)) return LT_IO_ERR_ARG;
  BitWriter w{out, cap};
  // child lookup: (code, byte) -> code in a 4096 x 256 table; an entry is valid only if its
  // generation is the current one, so a table reset (Clear) is one increment, not a 2 MB fill
  static thread_local std::vector<uint16_t> next_tl((size_t)4096 * 256, 0);
  static thread_local std::vector<uint32_t> gen_tl((size_t)4096 * 256, 0);
  static thread_local uint32_t cur_tl = 0;
  // one TLS lookup per call, not per byte (a thread_local access in a -fPIC library is a
  // __tls_get_addr call)
  uint16_t* const next = next_tl.data();
  uint32_t* const gen = gen_tl.data();
  uint32_t cur = cur_tl;
  struct Keep {
    uint32_t& dst;
    uint32_t& src;
    ~Keep() { dst = src; }
  } keep{cur_tl, cur};
  auto fresh = [&]() {
    if (++cur == 0) {  // wrapped: start over
      std::fill(gen, gen + (size_t)4096 * 256, 0u);
      cur = 1;
    }
  };
  fresh();
  int nbits = 9, free_ent = kFirst;
  w.put(kClear, nbits);
  if (n_in == 0) {
    w.put(kEoi, nbits);
    w.flush();
    return w.overflow ? LT_IO_ERR_SPACE : w.n;
  }
  int ent = in[0];
  for (int64_t k = 1; k < n_in; k++) {
    const int c = in[k];
    const size_t idx = (size_t)ent * 256 + c;
    if (gen[idx] == cur) {  // the string ent + c is in the table
      ent = next[idx];
      continue;
    }
    w.put(ent, nbits);
    next[idx] = (uint16_t)free_ent++;  // ent + c gets the next code
    gen[idx] = cur;
    ent = c;
    if (free_ent == (1 << kMaxBits) - 2) {  // table full (4094 codes): Clear, restart at 9 bits
      w.put(kClear, nbits);
      nbits = 9;
      free_ent = kFirst;
      fresh();
    } else if (free_ent > (1 << nbits) - 1) {
      nbits++;
    }
  }
  w.put(ent, nbits);
  free_ent++;
  if (free_ent == (1 << kMaxBits) - 2) {
    w.put(kClear, nbits);
    nbits = 9;
  } else if (free_ent > (1 << nbits) - 1) {
    nbits++;
  }
  w.put(kEoi, nbits);
  w.flush();
  return w.overflow ? LT_IO_ERR_SPACE : w.n;
}

// ---- whole images: every strip of a TIFF image decoded / encoded on a pool of threads ----------
// (ingest of a 7000 x 7000 x 30-year stack is 5.9 GB of int16 band samples: one Python call per
// 14 KB strip capped the job's parse step at ~2 Mpx/s)

}  // extern "C"

namespace {

// n items over `threads` workers pulling indices from one counter; the first error wins
template <class F>
int64_t pool_run(int64_t n, int threads, F fn) {
  std::atomic<int64_t> next(0), err(0);
  auto work = [&]() {
    for (;;) {
      const int64_t k = next.fetch_add(1);
      if (k >= n || err.load() != 0) return;
      const int64_t r = fn(k);
      if (r < 0) {
        int64_t z = 0;
        err.compare_exchange_strong(z, r);
      }
    }
  };
  const int t = (int)std::max<int64_t>(1, std::min<int64_t>(threads, n));
  std::vector<std::thread> ws;
  for (int i = 1; i < t; i++) ws.emplace_back(work);
  work();
  for (auto& w : ws) w.join();
  return err.load();
}

void bswap_samples(uint8_t* p, int64_t n, int bps) {
  for (int64_t i = 0; i < n; i++, p += bps) std::reverse(p, p + bps);
}

// TIFF Predictor 2 (horizontal differencing) undone / applied in place on `rows` rows of
// `width` pixels x `spp` interleaved samples of `bps` bytes (native byte order, integer wrap)
template <class T>
void pred2(uint8_t* buf, int64_t rows, int64_t width, int spp, bool undo) {
  T* a = (T*)buf;
  for (int64_t y = 0; y < rows; y++) {
    T* r = a + y * width * spp;
    if (undo) {
      for (int64_t x = spp; x < width * spp; x++) r[x] = (T)(r[x] + r[x - spp]);
    } else {
      for (int64_t x = width * spp - 1; x >= spp; x--) r[x] = (T)(r[x] - r[x - spp]);
    }
  }
}

void predictor2(uint8_t* buf, int64_t rows, int64_t width, int spp, int bps, bool undo) {
  switch (bps) {
    case 1: pred2<uint8_t>(buf, rows, width, spp, undo); break;
    case 2: pred2<uint16_t>(buf, rows, width, spp, undo); break;
    case 4: pred2<uint32_t>(buf, rows, width, spp, undo); break;
    default: pred2<uint64_t>(buf, rows, width, spp, undo); break;
  }
}

}  // namespace

extern "C" {

int64_t lt_tiff_decode_strips(const uint8_t* file, int64_t file_size, const uint64_t* offsets,
                              const uint64_t* counts, int64_t n_strips, int compression,
                              int predictor, int bps, int big_endian, int64_t width,
                              int64_t height, int bands, int planar, int64_t rows_per_strip,
                              uint8_t* out, int threads) {
  if (!file || !offsets || !counts || !out || width <= 0 || height <= 0 || bands <= 0 ||
      rows_per_strip <= 0 || !(bps == 1 || bps == 2 || bps == 4 || bps == 8))
    return LT_IO_ERR_ARG;
  if (compression != 1 && compression != 5) return LT_IO_ERR_ARG;
  if (predictor != 1 && predictor != 2) return LT_IO_ERR_ARG;
  const int spp = planar == 1 ? bands : 1;  // samples per pixel inside one strip
  const int64_t per_band = (height + rows_per_strip - 1) / rows_per_strip;
  if (n_strips < (planar == 1 ? per_band : per_band * bands)) return LT_IO_ERR_ARG;
  const int64_t plane = width * height * bps;  // one band of `out`
  return pool_run(n_strips, threads, [&](int64_t k) -> int64_t {
    const int64_t b = planar == 1 ? 0 : k / per_band, r = planar == 1 ? k : k % per_band;
    if (b >= bands || r >= per_band) return 0;  // extra strips past the image: ignored
    const int64_t y0 = r * rows_per_strip;
    const int64_t rows = std::min(rows_per_strip, height - y0);
    const int64_t size = rows * width * spp * bps;
    if (offsets[k] > (uint64_t)file_size || counts[k] > (uint64_t)file_size - offsets[k])
      return LT_IO_ERR_DATA;
    const uint8_t* src = file + offsets[k];
    static thread_local std::vector<uint8_t> tmp;
    // planar 2 without byte swap or predictor: straight into the band's rows
    const bool direct = spp == 1;
    uint8_t* dst = direct ? out + b * plane + y0 * width * bps : nullptr;
    if (!direct) {
      tmp.resize((size_t)size);
      dst = tmp.data();
    }
    if (compression == 5) {
      const int64_t n = lt_lzw_decode(src, (int64_t)counts[k], dst, size);
      if (n < 0) return n;
      if (n < size) memset(dst + n, 0, (size_t)(size - n));  // a short strip: zero-padded (libtiff)
    } else {
      const int64_t n = std::min<int64_t>(size, (int64_t)counts[k]);
      memcpy(dst, src, (size_t)n);
      if (n < size) memset(dst + n, 0, (size_t)(size - n));
    }
    if (big_endian && bps > 1) bswap_samples(dst, rows * width * spp, bps);
    if (predictor == 2) predictor2(dst, rows, width, spp, bps, true);
    if (!direct) {  // chunky: de-interleave the samples into the band planes
      for (int bb = 0; bb < bands; bb++) {
        uint8_t* o = out + bb * plane + y0 * width * bps;
        const uint8_t* i = dst + bb * bps;
        for (int64_t px = 0; px < rows * width; px++) memcpy(o + px * bps, i + px * spp * bps, bps);
      }
    }
    return 0;
  });
}

int64_t lt_tiff_encode_strips(const uint8_t* in, int bands, int64_t rows, int64_t cols, int bps,
                              int64_t rows_per_strip, int compression, int predictor, uint8_t* out,
                              int64_t cap, int64_t* strip_sizes, int threads) {
  if (!in || !out || !strip_sizes || bands <= 0 || rows <= 0 || cols <= 0 || rows_per_strip <= 0 ||
      !(bps == 1 || bps == 2 || bps == 4 || bps == 8))
    return LT_IO_ERR_ARG;
  if ((compression != 1 && compression != 5) || (predictor != 1 && predictor != 2))
    return LT_IO_ERR_ARG;
  const int64_t per_band = (rows + rows_per_strip - 1) / rows_per_strip;
  const int64_t n = per_band * bands;
  std::vector<std::vector<uint8_t>> enc((size_t)n);
  const int64_t rc = pool_run(n, threads, [&](int64_t k) -> int64_t {
    const int64_t b = k / per_band, y0 = (k % per_band) * rows_per_strip;
    const int64_t nr = std::min(rows_per_strip, rows - y0);
    const int64_t size = nr * cols * bps;
    const uint8_t* src = in + (b * rows + y0) * cols * bps;
    static thread_local std::vector<uint8_t> tmp;
    if (predictor == 2) {
      tmp.assign(src, src + size);
      predictor2(tmp.data(), nr, cols, 1, bps, false);
      src = tmp.data();
    }
    std::vector<uint8_t>& e = enc[(size_t)k];
    if (compression == 1) {
      e.assign(src, src + size);
      return 0;
    }
    e.resize((size_t)(size * 3 / 2 + 16));
    const int64_t m = lt_lzw_encode(src, size, e.data(), (int64_t)e.size());
    if (m < 0) return m;
    e.resize((size_t)m);
    return 0;
  });
  if (rc < 0) return rc;
  int64_t total = 0;
  for (int64_t k = 0; k < n; k++) {
    const int64_t m = (int64_t)enc[(size_t)k].size();
    if (total + m > cap) return LT_IO_ERR_SPACE;
    memcpy(out + total, enc[(size_t)k].data(), (size_t)m);
    strip_sizes[k] = m;
    total += m;
  }
  return total;
}

}  // extern "C"
