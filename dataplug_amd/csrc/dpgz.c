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
 * Streaming form (dpgz_stream_*): the same points while the object passes through in bounded pieces, each
 * point carrying its own window.  BGZF-style members (compressed size in the header) are inflated
 * independently on a thread pool (dpgz_bgzf_scan + dpgz_inflate_members, with dpgz_par.c's decoder).
 *
 * C ABI (declared in include/dpgz.h), no exceptions, int status (0 = ok).
 */
#include <pthread.h>
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

int dpgz_abi_version(void) { return 3; }

/* ------------------------------------------------------------------------------------------ streaming
 * The same access points, built while the object streams through in bounded pieces (FASTQ.gz objects far
 * larger than host memory, like the reference's 64 KiB writes into gztool's stdin, gzipped.py:62-83):
 * compressed bytes go in as they arrive, inflated bytes come out into the caller's (pinned) piece buffer,
 * and each point carries its own 32 KiB window (zlib's history at that block boundary, inflateGetDictionary)
 * and the inflated byte before it, so nothing behind the current piece has to be kept. */
struct dpgz_stream {
  z_stream z;
  int active;                 /* inside a member */
  int failed;
  uint64_t in_total;          /* compressed offset of the next input byte */
  uint64_t out_total;         /* inflated bytes produced so far */
  uint64_t span, last;
  uint64_t members;
  int32_t prev;               /* last inflated byte, -1 before any */
  dpgz_point_ex* pts;         /* points not yet taken */
  uint64_t npts, pcap;
  uint8_t* win;               /* their windows, concatenated */
  uint64_t nwin, wcap;
};

int dpgz_stream_new(uint64_t span, dpgz_stream** out) {
  if (!out) return DPGZ_ERR_INVALID;
  dpgz_stream* s = (dpgz_stream*)calloc(1, sizeof(dpgz_stream));
  if (!s) return DPGZ_ERR_MEMORY;
  s->span = span ? span : (1u << 20);
  s->prev = -1;
  *out = s;
  return DPGZ_OK;
}

void dpgz_stream_free(dpgz_stream* s) {
  if (!s) return;
  if (s->active) inflateEnd(&s->z);
  free(s->pts);
  free(s->win);
  free(s);
}

static int stream_point(dpgz_stream* s, uint64_t in_byte, uint32_t bits, uint32_t member) {
  if (grow((void**)&s->pts, &s->pcap, s->npts + 1, sizeof(dpgz_point_ex))) return -1;
  dpgz_point_ex* p = &s->pts[s->npts++];
  p->in_byte = in_byte;
  p->out_byte = s->out_total;
  p->bits = bits;
  p->member_start = member;
  p->prev_byte = s->prev;
  p->window_len = 0;
  if (!member) {
    if (grow((void**)&s->win, &s->wcap, s->nwin + 32768, 1)) return -1;
    uInt n = 0;
    if (inflateGetDictionary(&s->z, s->win + s->nwin, &n) != Z_OK) return -1;
    p->window_len = n;
    s->nwin += n;
  }
  s->last = s->out_total;
  return 0;
}

int dpgz_stream_inflate(dpgz_stream* s, const uint8_t* in, uint64_t in_len, int in_final, uint8_t* out,
                        uint64_t out_cap, uint64_t* consumed, uint64_t* produced, int* at_end) {
  if (!s || (!in && in_len) || (!out && out_cap) || !consumed || !produced || !at_end) return DPGZ_ERR_INVALID;
  if (s->failed) return s->failed;
  uint64_t ci = 0, po = 0;
  int rc = DPGZ_OK, stuck = 0;
  *at_end = 0;
  while (po < out_cap) {
    if (!s->active) {
      while (ci < in_len && in[ci] == 0) ++ci;          /* zero padding after a member (like gzip -d) */
      if (ci == in_len) {
        if (in_final) *at_end = 1;
        break;
      }
      memset(&s->z, 0, sizeof(s->z));
      if (inflateInit2(&s->z, 31) != Z_OK) { rc = DPGZ_ERR_ZLIB; break; }
      s->active = 1;
      if (stream_point(s, s->in_total + ci, 0, 1)) { rc = DPGZ_ERR_MEMORY; break; }
      ++s->members;
    }
    const uint64_t left = in_len - ci;
    s->z.next_in = (Bytef*)(in + ci);
    s->z.avail_in = (uInt)(left > 0x40000000ull ? 0x40000000ull : left);
    const uint64_t room = out_cap - po;
    s->z.next_out = out + po;
    s->z.avail_out = (uInt)(room > DPGZ_CHUNK ? DPGZ_CHUNK : room);
    const uInt ai = s->z.avail_in, ao = s->z.avail_out;
    const int zr = inflate(&s->z, Z_BLOCK);
    const uint64_t used = ai - s->z.avail_in, made = ao - s->z.avail_out;
    if (made) s->prev = out[po + made - 1];
    ci += used;
    po += made;
    s->out_total += made;
    if (zr == Z_STREAM_END) {
      inflateEnd(&s->z);
      s->active = 0;
      continue;
    }
    if (zr != Z_OK && zr != Z_BUF_ERROR) { rc = DPGZ_ERR_ZLIB; break; }
    if (zr == Z_BUF_ERROR || (!used && !made)) {
      if (ci == in_len) {                                  /* needs more input */
        if (in_final) rc = DPGZ_ERR_TRUNCATED;
        break;
      }
      if (po == out_cap) break;                            /* needs more room */
      if (++stuck > 1) { rc = DPGZ_ERR_ZLIB; break; }      /* no progress with input and room: corrupt */
    } else {
      stuck = 0;
    }
    if ((s->z.data_type & 128) && !(s->z.data_type & 64) && s->out_total - s->last >= s->span) {
      if (stream_point(s, s->in_total + ci, (uint32_t)(s->z.data_type & 7), 0)) { rc = DPGZ_ERR_MEMORY; break; }
    }
  }
  s->in_total += ci;
  *consumed = ci;
  *produced = po;
  if (rc != DPGZ_OK) s->failed = rc;
  return rc;
}

int dpgz_stream_take(dpgz_stream* s, dpgz_point_ex* pts, uint64_t max_pts, uint8_t* windows, uint64_t win_cap,
                     uint64_t* n_pts, uint64_t* n_win) {
  if (!s || !n_pts || !n_win) return DPGZ_ERR_INVALID;
  uint64_t n = s->npts < max_pts ? s->npts : max_pts, w = 0;
  for (uint64_t i = 0; i < n; ++i) w += s->pts[i].window_len;
  while (w > win_cap && n > 0) w -= s->pts[--n].window_len;
  if (n && (!pts || (w && !windows))) return DPGZ_ERR_INVALID;
  memcpy(pts, s->pts, n * sizeof(dpgz_point_ex));
  memcpy(windows, s->win, w);
  memmove(s->pts, s->pts + n, (s->npts - n) * sizeof(dpgz_point_ex));
  memmove(s->win, s->win + w, s->nwin - w);
  s->npts -= n;
  s->nwin -= w;
  *n_pts = n;
  *n_win = w;
  return DPGZ_OK;
}

int dpgz_stream_state(dpgz_stream* s, uint64_t* in_total, uint64_t* out_total, uint64_t* members, uint64_t* pending_pts,
                      uint64_t* pending_win) {
  if (!s) return DPGZ_ERR_INVALID;
  if (in_total) *in_total = s->in_total;
  if (out_total) *out_total = s->out_total;
  if (members) *members = s->members;
  if (pending_pts) *pending_pts = s->npts;
  if (pending_win) *pending_win = s->nwin;
  return DPGZ_OK;
}

/* ------------------------------------------------------------------------------------------ BGZF members
 * Members whose compressed size is in their header (the BGZF "BC" extra subfield: BSIZE + 1) and whose
 * inflated size is their ISIZE trailer can be inflated independently: one member per task on a thread pool,
 * each straight to its place in the output. */
int dpgz_bgzf_scan(const uint8_t* gz, uint64_t len, uint64_t* in_off, uint64_t* in_len, uint64_t* out_len,
                   uint64_t cap, uint64_t* n, uint64_t* used) {
  if ((!gz && len) || !n || !used) return DPGZ_ERR_INVALID;
  uint64_t p = 0, k = 0;
  while (k < cap) {
    while (p < len && gz[p] == 0) ++p;
    if (len - p < 18) break;
    const uint8_t* h = gz + p;
    if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) return DPGZ_ERR_ZLIB;   /* not BGZF */
    const uint64_t xlen = (uint64_t)h[10] | ((uint64_t)h[11] << 8);
    if (len - p < 12 + xlen) break;
    uint64_t bsize = 0;
    for (uint64_t q = 12; q + 4 <= 12 + xlen;) {
      const uint64_t slen = (uint64_t)h[q + 2] | ((uint64_t)h[q + 3] << 8);
      if (h[q] == 'B' && h[q + 1] == 'C' && slen == 2) bsize = ((uint64_t)h[q + 4] | ((uint64_t)h[q + 5] << 8)) + 1;
      q += 4 + slen;
    }
    if (!bsize) return DPGZ_ERR_ZLIB;
    if (len - p < bsize) break;                             /* member continues past this batch */
    const uint8_t* t = gz + p + bsize - 4;
    in_off[k] = p;
    in_len[k] = bsize;
    out_len[k] = (uint64_t)t[0] | ((uint64_t)t[1] << 8) | ((uint64_t)t[2] << 16) | ((uint64_t)t[3] << 24);
    ++k;
    p += bsize;
  }
  *n = k;
  *used = p;
  return DPGZ_OK;
}

typedef struct {
  const uint8_t* gz;
  const uint64_t *in_off, *in_len, *out_off, *out_len;
  uint8_t* out;
  uint64_t n;
  uint64_t next;              /* next member to take (atomic) */
  int rc;
} members_job;

/* dpgz_par.c's decoder for one whole member (faster than zlib's inflate on these CPUs; CRC-checked), its
 * per-thread state, and its process-wide thread pool */
int dpgz__member(const uint8_t* gz, uint64_t len, uint8_t* out, uint64_t out_len, void** scratch);
void* dpgz__scratch_get(void);
void dpgz__scratch_put(void* scratch);
void dpgz__global_for(int threads, int n, void (*fn)(void*, int), void* arg);

#define MEMBERS_PER_ITEM 1u
static void members_item(void* arg, int item) {
  members_job* j = (members_job*)arg;
  void* scratch = dpgz__scratch_get();
  const uint64_t i0 = (uint64_t)item * MEMBERS_PER_ITEM;
  for (uint64_t i = i0; i < j->n && i < i0 + MEMBERS_PER_ITEM; ++i) {
    if (__atomic_load_n(&j->rc, __ATOMIC_RELAXED)) break;
    const int rc = dpgz__member(j->gz + j->in_off[i], j->in_len[i], j->out + j->out_off[i], j->out_len[i], &scratch);
    if (rc) {
      int zero = 0;
      __atomic_compare_exchange_n(&j->rc, &zero, rc, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED);
    }
  }
  dpgz__scratch_put(scratch);
}

int dpgz_inflate_members(const uint8_t* gz, const uint64_t* in_off, const uint64_t* in_len, const uint64_t* out_off,
                         const uint64_t* out_len, uint64_t n, uint8_t* out, int threads) {
  if ((!gz || !in_off || !in_len || !out_off || !out_len || !out) && n) return DPGZ_ERR_INVALID;
  members_job j = {gz, in_off, in_len, out_off, out_len, out, n, 0, DPGZ_OK};
  const uint64_t items = (n + MEMBERS_PER_ITEM - 1) / MEMBERS_PER_ITEM;
  if (items > 0x7FFFFFFFull) return DPGZ_ERR_INVALID;
  if (threads <= 1 || items <= 1) {
    for (uint64_t k = 0; k < items; ++k) members_item(&j, (int)k);
  } else {
    dpgz__global_for(threads, (int)items, members_item, &j);
  }
  return j.rc;
}
