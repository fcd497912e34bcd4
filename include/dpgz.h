/*
 * dpgz.h — C ABI of libdpgz.so: gzip access-point index for random access into GZipText / FASTQGZip
 * objects (replaces the gztool -i/-x index of dataplug/formats/compressed/gzipped.py:46-153 and the
 * gztool -n/-L resume of GZipTextSlice._lines_iterator, gzipped.py:268-354).  Host code (zlib).
 */
#ifndef DPGZ_H
#define DPGZ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPGZ_OK 0
#define DPGZ_ERR_INVALID 1
#define DPGZ_ERR_MEMORY 2
#define DPGZ_ERR_ZLIB 3        /* corrupt deflate / gzip data */
#define DPGZ_ERR_TRUNCATED 4   /* the input ends inside a member */

typedef struct {
  uint64_t in_byte;        /* compressed offset: member start, or the byte after the block start */
  uint64_t out_byte;       /* uncompressed offset of the point */
  uint32_t bits;           /* bits of byte in_byte-1 that belong to the block (0..7) */
  uint32_t member_start;   /* 1: a gzip member starts at in_byte (no history needed) */
} dpgz_point;

typedef struct {
  uint8_t* out;            /* the whole inflated stream (malloc'ed) */
  uint64_t out_len;
  dpgz_point* points;      /* access points in increasing order */
  uint64_t n_points;
  uint64_t members;        /* gzip members seen */
} dpgz_result;

int dpgz_abi_version(void);
/* Inflate a (multi-member) gzip stream; access points every `span` output bytes at deflate block
 * boundaries plus every member start.  out_hint: expected inflated size (0: guess). */
int dpgz_build(const uint8_t* gz, uint64_t gz_len, uint64_t span, uint64_t out_hint, dpgz_result** result);
void dpgz_free(dpgz_result* result);

#ifdef __cplusplus
}
#endif
#endif
