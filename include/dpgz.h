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

typedef struct {
  uint64_t in_byte;        /* as dpgz_point */
  uint64_t out_byte;
  uint32_t bits;
  uint32_t member_start;
  int32_t prev_byte;       /* the inflated byte before out_byte, -1 at 0 */
  uint32_t window_len;     /* bytes of this point's window in the blob dpgz_stream_take returns (0: member start) */
} dpgz_point_ex;

typedef struct dpgz_stream dpgz_stream;

int dpgz_abi_version(void);
/* Inflate a (multi-member) gzip stream; access points every `span` output bytes at deflate block
 * boundaries plus every member start.  out_hint: expected inflated size (0: guess). */
int dpgz_build(const uint8_t* gz, uint64_t gz_len, uint64_t span, uint64_t out_hint, dpgz_result** result);
void dpgz_free(dpgz_result* result);

/* Streaming build: feed compressed bytes as they arrive (in_final = 1 with the last ones), get inflated
 * bytes into `out` (at most out_cap; the call returns when the input is used up, the output is full or the
 * stream ends: *at_end).  Access points found on the way queue up with their 32 KiB windows until taken. */
int dpgz_stream_new(uint64_t span, dpgz_stream** out);
void dpgz_stream_free(dpgz_stream* s);
int dpgz_stream_inflate(dpgz_stream* s, const uint8_t* in, uint64_t in_len, int in_final, uint8_t* out,
                        uint64_t out_cap, uint64_t* consumed, uint64_t* produced, int* at_end);
int dpgz_stream_take(dpgz_stream* s, dpgz_point_ex* pts, uint64_t max_pts, uint8_t* windows, uint64_t win_cap,
                     uint64_t* n_pts, uint64_t* n_win);
int dpgz_stream_state(dpgz_stream* s, uint64_t* in_total, uint64_t* out_total, uint64_t* members,
                      uint64_t* pending_pts, uint64_t* pending_win);

/* BGZF-style members (FEXTRA "BC" subfield = compressed size - 1; ISIZE = inflated size): list the complete
 * members at the start of `gz` (*used = bytes they span; DPGZ_ERR_ZLIB if a member is not of this kind),
 * then inflate any of them independently on `threads` threads, each to out + out_off[i]. */
int dpgz_bgzf_scan(const uint8_t* gz, uint64_t len, uint64_t* in_off, uint64_t* in_len, uint64_t* out_len,
                   uint64_t cap, uint64_t* n, uint64_t* used);
int dpgz_inflate_members(const uint8_t* gz, const uint64_t* in_off, const uint64_t* in_len, const uint64_t* out_off,
                         const uint64_t* out_len, uint64_t n, uint8_t* out, int threads);

/* Parallel inflate of one gzip stream (dpgz_par.c): speculative deflate block starts per region, 16-bit
 * marker windows resolved in order, every member's CRC-32 / ISIZE checked.  Feed compressed bytes (the
 * engine inflates a batch once 2 x threads x 1 MiB are pending, or everything with in_final), read the inflated
 * bytes in order, take the access points (those of dpgz_stream, with windows) up to an output offset.
 * dpgz_par_state fills stats[14]: compressed bytes consumed, inflated bytes produced, members, inflated
 * bytes not read, points pending, window bytes pending, stream ended, batches, region starts rejected, then
 * nanoseconds spent in the block search (0: now part of each region's decode task), the speculative decode,
 * the window chain, marker resolution + CRC, and the
 * in-order bookkeeping (CRC combine, access points) of all batches. */
typedef struct dpgz_par dpgz_par;
int dpgz_par_new(uint64_t span, int threads, dpgz_par** out);
void dpgz_par_free(dpgz_par* s);
int dpgz_par_set_region(dpgz_par* s, uint64_t bytes);   /* compressed bytes per region (default 2 MiB) */
int dpgz_par_feed(dpgz_par* s, const uint8_t* in, uint64_t in_len, int in_final);
int dpgz_par_read(dpgz_par* s, uint8_t* out, uint64_t cap, uint64_t* n);
int dpgz_par_take(dpgz_par* s, uint64_t out_limit, dpgz_point_ex* pts, uint64_t max_pts, uint8_t* windows,
                  uint64_t win_cap, uint64_t* n_pts, uint64_t* n_win);
int dpgz_par_state(dpgz_par* s, uint64_t* stats);

#ifdef __cplusplus
}
#endif
#endif
