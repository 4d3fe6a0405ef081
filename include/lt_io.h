/*
 * lt_io.h — host codecs of the raster IO around the hot path (land_trendr_amd/liblt_io.so).
 *
 * The reference reads and writes GeoTIFFs through GDAL: ds2array (/root/reference/utils.py:
 * 272-282) decodes whatever compression the input rasters carry, array2raster (utils.py:374-412)
 * writes every output raster with COMPRESS=LZW (utils.py:386). GDAL is absent here; these are the
 * LZW halves of that (Deflate goes through zlib). Plain pointers and sizes; the caller owns both
 * buffers. Return: bytes written (>= 0) or a negative LT_IO_ERR_*.
 */
#ifndef LT_IO_H
#define LT_IO_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { LT_IO_ERR_ARG = -1, LT_IO_ERR_DATA = -2, LT_IO_ERR_SPACE = -3 };

/* One TIFF LZW strip or tile (Compression = 5) -> its raw bytes (at most cap; bytes of out past
 * the returned count may be overwritten, never past cap). */
int64_t lt_lzw_decode(const uint8_t* in, int64_t n_in, uint8_t* out, int64_t cap);
/* Raw bytes -> one TIFF LZW strip (libtiff's code stream: Clear first, 9..12-bit codes, early
 * change, Clear when the table is full). cap >= n_in * 3 / 2 + 16 always suffices. */
int64_t lt_lzw_encode(const uint8_t* in, int64_t n_in, uint8_t* out, int64_t cap);

/* Every strip of one strip-organised TIFF image decoded on `threads` threads into `out`, the
 * [bands, height, width] samples in native byte order (what ds2array gives per band,
 * /root/reference/utils.py:272-282): compression 1 or 5, predictor 1 or 2 (integer horizontal
 * differencing, undone with wrap), planar 1 (chunky: de-interleaved here) or 2; a short strip is
 * zero-padded as libtiff pads it. Strip k of `file` is file[offsets[k] : offsets[k] + counts[k]].
 * Returns 0 or a negative LT_IO_ERR_*. */
int64_t lt_tiff_decode_strips(const uint8_t* file, int64_t file_size, const uint64_t* offsets,
                              const uint64_t* counts, int64_t n_strips, int compression,
                              int predictor, int bps, int big_endian, int64_t width,
                              int64_t height, int bands, int planar, int64_t rows_per_strip,
                              uint8_t* out, int threads);
/* [bands, rows, cols] samples (little-endian) -> the strips of a planar-2 TIFF image, band by
 * band, rows_per_strip rows each, compression 1 or 5 (array2raster's COMPRESS=LZW,
 * utils.py:386), predictor 1 or 2, encoded on `threads` threads and laid back to back in `out`
 * (cap bytes); strip_sizes[k] gets each strip's length. Returns the total bytes or a negative
 * LT_IO_ERR_*. */
int64_t lt_tiff_encode_strips(const uint8_t* in, int bands, int64_t rows, int64_t cols, int bps,
                              int64_t rows_per_strip, int compression, int predictor, uint8_t* out,
                              int64_t cap, int64_t* strip_sizes, int threads);

#ifdef __cplusplus
}
#endif
#endif
