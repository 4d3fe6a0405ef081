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
  uint32_t acc = 0;
  int nacc = 0;
  bool overflow = false;
  void put(int code, int nbits) {
    acc = (acc << nbits) | (uint32_t)code;
    nacc += nbits;
    while (nacc >= 8) {
      nacc -= 8;
      byte((uint8_t)(acc >> nacc));
    }
    acc &= (1u << nacc) - 1u;
  }
  void byte(uint8_t b) {
    if (n < cap) out[n] = b;
    else overflow = true;
    n++;
  }
  void flush() {
    if (nacc > 0) byte((uint8_t)(acc << (8 - nacc)));
    nacc = 0;
    acc = 0;
  }
};

}  // namespace

extern "C" {

int64_t lt_lzw_decode(const uint8_t* in, int64_t n_in, uint8_t* out, int64_t cap) {
  if (!in || n_in < 0 || (cap > 0 && !out)) return LT_IO_ERR_ARG;
  // string table: prefix code, last byte, length, first byte
  static thread_local uint16_t prefix[4096];
  static thread_local uint8_t last[4096], first[4096];
  static thread_local uint16_t len[4096];
  for (int c = 0; c < 256; c++) {
    prefix[c] = 0xFFFF;
    last[c] = first[c] = (uint8_t)c;
    len[c] = 1;
  }
  int nbits = 9, free_ent = kFirst, old = -1;
  int64_t n_out = 0, byte_pos = 0;
  // bit reader: whole bytes into a 64-bit buffer, codes taken from its top (MSB first); a code
  // the remaining input cannot fill ends the strip
  uint64_t bitbuf = 0;
  int nbuf = 0;
  auto get = [&](int nb) -> int {
    while (nbuf < nb) {
      if (byte_pos >= n_in) return -1;
      bitbuf = (bitbuf << 8) | in[byte_pos++];
      nbuf += 8;
    }
    nbuf -= nb;
    return (int)((bitbuf >> nbuf) & ((1u << nb) - 1u));
  };
  auto emit = [&](int code) -> bool {
    const int L = len[code];
    if (n_out + L > cap) return false;
    int c = code;
    for (int k = L - 1; k >= 0; k--) {
      out[n_out + k] = last[c];
      c = prefix[c];
    }
    n_out += L;
    return true;
  };
  for (;;) {
    int code = get(nbits);
    if (code < 0 || code == kEoi) break;  // a strip may end without EOI (libtiff tolerates it)
    if (code == kClear) {
      nbits = 9;
      free_ent = kFirst;
      code = get(nbits);
      if (code < 0 || code == kEoi) break;
      if (code >= 256) return LT_IO_ERR_DATA;
      if (!emit(code)) return LT_IO_ERR_SPACE;
      old = code;
      continue;
    }
    if (old < 0) {  // data must start with a Clear code or a literal
      if (code >= 256) return LT_IO_ERR_DATA;
      if (!emit(code)) return LT_IO_ERR_SPACE;
      old = code;
      continue;
    }
    if (code < free_ent && code != kClear && code != kEoi) {
      if (!emit(code)) return LT_IO_ERR_SPACE;
      if (free_ent < 4096) {
        prefix[free_ent] = (uint16_t)old;
        last[free_ent] = first[code];
        first[free_ent] = first[old];
        len[free_ent] = (uint16_t)(len[old] + 1);
        free_ent++;
      }
    } else if (code == free_ent && free_ent < 4096) {
      prefix[free_ent] = (uint16_t)old;
      last[free_ent] = first[old];
      first[free_ent] = first[old];
      len[free_ent] = (uint16_t)(len[old] + 1);
      free_ent++;
      if (!emit(code)) return LT_IO_ERR_SPACE;
    } else {
      return LT_IO_ERR_DATA;
    }
    old = code;
    if (free_ent >= (1 << nbits) - 1 && nbits < kMaxBits) nbits++;
  }
  return n_out;
}

int64_t lt_lzw_encode(const uint8_t* in, int64_t n_in, uint8_t* out, int64_t cap) {
  if (!in || n_in < 0 || (cap > 0 && !out)) return LT_IO_ERR_ARG;
  BitWriter w{out, cap};
  // child lookup: (code, byte) -> code in a 4096 x 256 table; an entry is valid only if its
  // generation is the current one, so a table reset (Clear) is one increment, not a 2 MB fill
  static thread_local std::vector<uint16_t> next((size_t)4096 * 256, 0);
  static thread_local std::vector<uint32_t> gen((size_t)4096 * 256, 0);
  static thread_local uint32_t cur = 0;
  auto fresh = [&]() {
    if (++cur == 0) {  // wrapped: start over
      std::fill(gen.begin(), gen.end(), 0u);
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
