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

}  // extern "C"
