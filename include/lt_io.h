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

/* One TIFF LZW strip or tile (Compression = 5) -> its raw bytes (at most cap). */
int64_t lt_lzw_decode(const uint8_t* in, int64_t n_in, uint8_t* out, int64_t cap);
/* Raw bytes -> one TIFF LZW strip (libtiff's code stream: Clear first, 9..12-bit codes, early
 * change, Clear when the table is full). cap >= n_in * 3 / 2 + 16 always suffices. */
int64_t lt_lzw_encode(const uint8_t* in, int64_t n_in, uint8_t* out, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif
