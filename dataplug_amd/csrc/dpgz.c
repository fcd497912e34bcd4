/*
 * dpgz.c — host-side gzip access-point index (libdpgz.so), the random-access half of the GZipText /
 * FASTQGZip path.
 *
 * The reference builds this with gztool 1.4.3 (dataplug/formats/compressed/gzipped.py:46-153: a window
 * table of (compressed_byte, uncompressed_byte, line_number, window_size, window_offset) and a binary
 * index that lets gztool resume inflating mid-stream).  Here one pass of zlib inflate with Z_BLOCK
 * stops at every deflate block boundary; every `span` output bytes a boundary becomes an access point
 * (compressed byte, the number of bits of the previous byte that belong to the block, uncompressed
 * byte), and every gzip member start is one too.  The 32 KiB history a point needs is the inflated
 * output just before it, which the caller keeps (the whole inflated stream is returned — it is also
 * what the GPU newline scan runs over).
 *
 * Resuming at a point needs the bit offset: the Python side shifts the compressed bytes so the block
 * starts at bit 0 and inflates raw with the window as dictionary (no inflatePrime needed there).
 *
 * C ABI (declared in include/dpgz.h), no exceptions, int status (0 = ok).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "../../include/dpgz.h"

#define DPGZ_CHUNK (1u << 20)

static int grow(void** p, uint64_t* cap, uint64_t need, uint64_t elem) {
  if (need <= *cap) return 0;
  uint64_t c = *cap ? *cap : 1024;
  while (c < need) c *= 2;
  void* q = realloc(*p, c * elem);
  if (!q) return -1;
  *p = q;
  *cap = c;
  return 0;
}

static int add_point(dpgz_result* r, uint64_t* pcap, uint64_t in, uint32_t bits, uint64_t out, uint32_t member) {
  if (grow((void**)&r->points, pcap, r->n_points + 1, sizeof(dpgz_point))) return -1;
  dpgz_point* p = &r->points[r->n_points++];
  p->in_byte = in;
  p->out_byte = out;
  p->bits = bits;
  p->member_start = member;
  return 0;
}

int dpgz_build(const uint8_t* gz, uint64_t gz_len, uint64_t span, uint64_t out_hint, dpgz_result** result) {
  if (!gz || !result) return DPGZ_ERR_INVALID;
  *result = NULL;
  dpgz_result* r = (dpgz_result*)calloc(1, sizeof(dpgz_result));
  if (!r) return DPGZ_ERR_MEMORY;
  uint64_t ocap = out_hint ? out_hint : (gz_len * 4 + 4096), pcap = 0;
  r->out = (uint8_t*)malloc(ocap);
  if (!r->out) { free(r); return DPGZ_ERR_MEMORY; }

  z_stream s;
  memset(&s, 0, sizeof(s));
  uint64_t pos = 0;               /* compressed bytes consumed before the current member */
  uint64_t last = 0;              /* output offset of the last access point */
  int rc = DPGZ_OK;
  while (pos < gz_len) {
    /* a gzip member starts here */
    if (inflateInit2(&s, 31) != Z_OK) { rc = DPGZ_ERR_ZLIB; break; }
    if (add_point(r, &pcap, pos, 0, r->out_len, 1)) { rc = DPGZ_ERR_MEMORY; inflateEnd(&s); break; }
    last = r->out_len;
    s.next_in = (Bytef*)(gz + pos);
    uint64_t left = gz_len - pos;
    s.avail_in = (uInt)(left > 0x40000000ull ? 0x40000000ull : left);
    uint64_t fed = s.avail_in;
    int zr = Z_OK;
    for (;;) {
      if (s.avail_in == 0 && fed < left) {
        const uint64_t more = left - fed > 0x40000000ull ? 0x40000000ull : left - fed;
        s.next_in = (Bytef*)(gz + pos + fed);
        s.avail_in = (uInt)more;
        fed += more;
      }
      if (r->out_len + DPGZ_CHUNK > ocap) {
        uint64_t nc = ocap * 2;
        while (nc < r->out_len + DPGZ_CHUNK) nc *= 2;
        uint8_t* q = (uint8_t*)realloc(r->out, nc);
        if (!q) { rc = DPGZ_ERR_MEMORY; break; }
        r->out = q;
        ocap = nc;
      }
      s.next_out = r->out + r->out_len;
      s.avail_out = DPGZ_CHUNK;
      zr = inflate(&s, Z_BLOCK);
      r->out_len += DPGZ_CHUNK - s.avail_out;
      if (zr == Z_STREAM_END) break;
      if (zr != Z_OK && zr != Z_BUF_ERROR) { rc = DPGZ_ERR_ZLIB; break; }
      if (zr == Z_BUF_ERROR && s.avail_in == 0 && fed >= left) { rc = DPGZ_ERR_TRUNCATED; break; }
      /* at the end of a deflate block header that is not the last block: a possible access point */
      if ((s.data_type & 128) && !(s.data_type & 64) && r->out_len - last >= span) {
        const uint64_t consumed = pos + (uint64_t)(s.next_in - (gz + pos));
        if (add_point(r, &pcap, consumed, (uint32_t)(s.data_type & 7), r->out_len, 0)) { rc = DPGZ_ERR_MEMORY; break; }
        last = r->out_len;
      }
    }
    const uint64_t consumed = pos + (uint64_t)(s.next_in - (gz + pos));
    inflateEnd(&s);
    if (rc != DPGZ_OK) break;
    pos = consumed;
    /* trailing zero padding after the last member is tolerated (like gzip -d) */
    while (pos < gz_len && gz[pos] == 0) ++pos;
  }
  if (rc != DPGZ_OK) {
    dpgz_free(r);
    return rc;
  }
  r->members = 0;
  for (uint64_t i = 0; i < r->n_points; ++i) r->members += r->points[i].member_start;
  *result = r;
  return DPGZ_OK;
}

void dpgz_free(dpgz_result* r) {
  if (!r) return;
  free(r->out);
  free(r->points);
  free(r);
}

int dpgz_abi_version(void) { return 1; }
