/*
 * dpgz_par.c — parallel inflate of ONE gzip stream (part of libdpgz.so).
 *
 * A plain gzip member is a single deflate stream: zlib (and gztool in the reference,
 * dataplug/formats/compressed/gzipped.py:46-153) inflate it on one core.  This engine inflates it on
 * `threads` cores, one batch of compressed bytes at a time:
 *
 *  1. the batch is cut into regions; each thread looks for the first deflate block start in its region:
 *     a dynamic-Huffman header that passes every structural check (BFINAL 0, BTYPE 2, HLIT <= 29,
 *     HDIST <= 29, a complete code-length code, complete literal/length code holding an end-of-block code,
 *     a valid distance code) and whose block then decodes to its end-of-block code;
 *  2. each thread decodes from its start to the next region's start into 16-bit symbols: a byte, or a
 *     marker 256 + j standing for byte j of the (not yet known) 32 KiB before its start;
 *  3. region i is kept only if region i-1's decode stopped exactly at region i's start (a false start makes
 *     region i-1 run past it; the batch then ends where region i-1 stopped and the next batch goes on);
 *  4. the windows are resolved in order (the last 32 KiB of each region only), then every region's markers
 *     are replaced in parallel, and each member's CRC-32 and ISIZE are checked against its trailer, so a
 *     wrong speculative decode cannot pass silently.
 *
 * The access points are those of dpgz_stream (the first block start at least `span` inflated bytes after the
 * previous point, and every member start) with the same windows.  A batch ends at a block start or a member
 * boundary; the compressed bytes from there on wait for the next batch.  Host memory: the pending compressed
 * bytes, 2 bytes per inflated byte of one batch, and the resolved output until it is read.
 */
#include <pthread.h>
#include <time.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "../../include/dpgz.h"

#define WIN 32768u
#define LBITS 10
#define DBITS 8
#define LTAB (1024 + 288 * 32)
#define DTAB (256 + 30 * 128)
#define CLTAB 128
#define E_SUB 0x100000u
#define REGION_MIN (1u << 20)           /* compressed bytes per region, at least (default) */
#define NONE UINT64_MAX

enum { K_BLOCK = 0, K_HEADER = 1, K_END = 2 };           /* what starts at a stop position */
enum { D_OK = 0, D_BAD = -1, D_INPUT = -2, D_MEM = -3, D_TRUNC = -4 };
enum { EV_BLOCK = 0, EV_MSTART = 1, EV_MEND = 2 };

/* ------------------------------------------------------------------------------------------ tables */
static const uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                      35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

static uint32_t rev_bits(uint32_t c, int n) {
  uint32_t r = 0;
  for (int i = 0; i < n; ++i) r = (r << 1) | ((c >> i) & 1u);
  return r;
}

/* Canonical Huffman lookup.  Entry: symbol | bits << 16 (bits 0: no such code), or E_SUB | offset |
 * subbits << 24 for a second-level table indexed by the next subbits bits (its entries hold the bits
 * beyond the first pbits).  -1 if the lengths over-subscribe the code or leave it incomplete (a code of
 * at most one symbol is accepted where allow_single, as zlib does for distances). */
static int build_table(uint32_t* tab, int cap, const uint8_t* lens, int n, int pbits, int allow_single) {
  int count[16] = {0};
  for (int i = 0; i < n; ++i) count[lens[i]]++;
  count[0] = 0;
  int left = 1, total = 0;
  for (int l = 1; l <= 15; ++l) {
    left <<= 1;
    left -= count[l];
    if (left < 0) return -1;
    total += count[l];
  }
  if (left > 0 && !(allow_single && total <= 1)) return -1;
  int next[16];
  int code = 0;
  next[0] = 0;
  for (int l = 1; l <= 15; ++l) {
    code = (code + count[l - 1]) << 1;
    next[l] = code;
  }
  const int psize = 1 << pbits;
  memset(tab, 0, sizeof(uint32_t) * (size_t)psize);
  uint8_t subbits[1024];
  memset(subbits, 0, (size_t)psize);
  int nx[16];
  memcpy(nx, next, sizeof(nx));
  for (int s = 0; s < n; ++s) {
    const int l = lens[s];
    if (l > pbits) {
      const uint32_t r = rev_bits((uint32_t)nx[l]++, l);
      const uint32_t p = r & (uint32_t)(psize - 1);
      if (l - pbits > subbits[p]) subbits[p] = (uint8_t)(l - pbits);
    }
  }
  int off = psize;
  for (int p = 0; p < psize; ++p) {
    if (!subbits[p]) continue;
    const int sz = 1 << subbits[p];
    if (off + sz > cap) return -1;
    memset(tab + off, 0, sizeof(uint32_t) * (size_t)sz);
    tab[p] = E_SUB | (uint32_t)off | ((uint32_t)subbits[p] << 24);
    off += sz;
  }
  memcpy(nx, next, sizeof(nx));
  for (int s = 0; s < n; ++s) {
    const int l = lens[s];
    if (!l) continue;
    const uint32_t r = rev_bits((uint32_t)nx[l]++, l);
    if (l <= pbits) {
      for (uint32_t i = r; i < (uint32_t)psize; i += 1u << l) tab[i] = (uint32_t)s | ((uint32_t)l << 16);
    } else {
      const uint32_t e = tab[r & (uint32_t)(psize - 1)];
      const uint32_t base = e & 0xFFFFu, sb = (e >> 24) & 15u;
      for (uint32_t i = r >> pbits; i < (1u << sb); i += 1u << (l - pbits))
        tab[base + i] = (uint32_t)s | ((uint32_t)(l - pbits) << 16);
    }
  }
  return 0;
}

typedef struct {
  uint32_t lit[LTAB];
  uint32_t dist[DTAB];
} Tables;

static Tables g_fixed;
static pthread_once_t g_fixed_once = PTHREAD_ONCE_INIT;
static void fixed_init(void) {
  uint8_t l[320];
  for (int i = 0; i < 144; ++i) l[i] = 8;
  for (int i = 144; i < 256; ++i) l[i] = 9;
  for (int i = 256; i < 280; ++i) l[i] = 7;
  for (int i = 280; i < 288; ++i) l[i] = 8;
  for (int i = 0; i < 32; ++i) l[288 + i] = 5;         /* distance codes 30, 31 exist but are invalid */
  build_table(g_fixed.lit, LTAB, l, 288, LBITS, 0);
  build_table(g_fixed.dist, DTAB, l + 288, 32, DBITS, 1);
}

/* ------------------------------------------------------------------------------------------ CRC-32
 * gzip's CRC-32 by carry-less multiplication (x86-64 PCLMULQDQ): four 128-bit lanes folded 64 bytes at a
 * time with x^(512±32) mod P, folded to one lane with x^(128±32) mod P, reduced 128 -> 64 -> 32 bits
 * (Barrett); the bit-reflected constants of P = 0x104C11DB7.  zlib's table method for tails and for CPUs
 * without the instruction (checked once). */
#if defined(__x86_64__)
#include <immintrin.h>
__attribute__((target("pclmul,sse4.1"))) static uint32_t crc_fold(uint32_t state, const uint8_t* p, uint64_t n) {
  /* state: the raw register (~crc); n >= 64, a multiple of 16 */
  const __m128i k512 = _mm_set_epi64x(0x01c6e41596ll, 0x0154442bd4ll);
  const __m128i k128 = _mm_set_epi64x(0x00ccaa009ell, 0x01751997d0ll);
  const __m128i k64 = _mm_set_epi64x(0, 0x0163cd6124ll);
  const __m128i pmu = _mm_set_epi64x(0x01f7011641ll, 0x01db710641ll);
  const __m128i lo32 = _mm_setr_epi32(-1, 0, -1, 0);
  __m128i a = _mm_xor_si128(_mm_loadu_si128((const __m128i*)p), _mm_cvtsi32_si128((int)state));
  __m128i b = _mm_loadu_si128((const __m128i*)(p + 16));
  __m128i c = _mm_loadu_si128((const __m128i*)(p + 32));
  __m128i d = _mm_loadu_si128((const __m128i*)(p + 48));
  p += 64;
  n -= 64;
  for (; n >= 64; p += 64, n -= 64) {
    const __m128i a1 = _mm_clmulepi64_si128(a, k512, 0x11), a0 = _mm_clmulepi64_si128(a, k512, 0x00);
    const __m128i b1 = _mm_clmulepi64_si128(b, k512, 0x11), b0 = _mm_clmulepi64_si128(b, k512, 0x00);
    const __m128i c1 = _mm_clmulepi64_si128(c, k512, 0x11), c0 = _mm_clmulepi64_si128(c, k512, 0x00);
    const __m128i d1 = _mm_clmulepi64_si128(d, k512, 0x11), d0 = _mm_clmulepi64_si128(d, k512, 0x00);
    a = _mm_xor_si128(_mm_xor_si128(a1, a0), _mm_loadu_si128((const __m128i*)p));
    b = _mm_xor_si128(_mm_xor_si128(b1, b0), _mm_loadu_si128((const __m128i*)(p + 16)));
    c = _mm_xor_si128(_mm_xor_si128(c1, c0), _mm_loadu_si128((const __m128i*)(p + 32)));
    d = _mm_xor_si128(_mm_xor_si128(d1, d0), _mm_loadu_si128((const __m128i*)(p + 48)));
  }
#define FOLD128(x, next) _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, k128, 0x11), \
                                                     _mm_clmulepi64_si128(x, k128, 0x00)), next)
  a = FOLD128(a, b);
  a = FOLD128(a, c);
  a = FOLD128(a, d);
  for (; n >= 16; p += 16, n -= 16) a = FOLD128(a, _mm_loadu_si128((const __m128i*)p));
#undef FOLD128
  /* 128 -> 64 bits */
  __m128i t = _mm_clmulepi64_si128(a, k128, 0x10);
  a = _mm_xor_si128(_mm_srli_si128(a, 8), t);
  t = _mm_srli_si128(a, 4);
  a = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(a, lo32), k64, 0x00), t);
  /* Barrett: 64 -> 32 bits */
  t = _mm_clmulepi64_si128(_mm_and_si128(a, lo32), pmu, 0x10);
  t = _mm_clmulepi64_si128(_mm_and_si128(t, lo32), pmu, 0x00);
  a = _mm_xor_si128(a, t);
  return (uint32_t)_mm_extract_epi32(a, 1);
}
static int g_pclmul = -1;
#endif

static uint32_t crc32_fast(uint32_t crc, const uint8_t* p, uint64_t n) {
#if defined(__x86_64__)
  if (g_pclmul < 0) g_pclmul = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
  if (g_pclmul && n >= 64) {
    const uint64_t m = n & ~15ull;
    crc = ~crc_fold(~crc, p, m);
    p += m;
    n -= m;
  }
#endif
  while (n > 0) {                                       /* zlib: uInt lengths */
    const uInt k = n > (1u << 30) ? (1u << 30) : (uInt)n;
    crc = (uint32_t)crc32(crc, p, k);
    p += k;
    n -= k;
  }
  return crc;
}

/* ------------------------------------------------------------------------------------------ bit input */
/* >= 57 valid bits from bit position pos (zeros past the end of the input). */
static inline uint64_t peek_at(const uint8_t* buf, uint64_t nbytes, uint64_t pos) {
  const uint64_t by = pos >> 3;
  uint64_t v = 0;
  if (by + 8 <= nbytes) {
    memcpy(&v, buf + by, 8);
  } else {
    for (uint64_t i = 0; by + i < nbytes && i < 8; ++i) v |= (uint64_t)buf[by + i] << (8 * i);
  }
  return v >> (pos & 7);
}

/* ------------------------------------------------------------------------------------------ decoding */
typedef struct {
  uint64_t bit;               /* stream bit position (relative to the batch buffer) */
  uint64_t out;               /* output index in the region's buffer (the WIN prefix included) */
  uint32_t kind;              /* EV_* */
  uint32_t crc;               /* EV_MEND: the trailer's CRC-32 */
  uint64_t isize;             /* EV_MEND: the trailer's ISIZE */
} Ev;

typedef struct {
  /* input of the decode */
  uint64_t start;             /* bit position */
  int start_kind;             /* K_BLOCK or K_HEADER */
  uint64_t stop_at;           /* stop at this block start (NONE: run to the end of the input) */
  uint64_t stop_after;        /* with stop_at NONE: stop at the first block start at or past this bit */
  uint64_t floor0;            /* lowest buffer index a back-reference may reach at the start */
  /* output */
  uint16_t* o;                /* [0, WIN): the window (bytes or markers), then the output */
  uint64_t n, cap;
  uint64_t floor;             /* lowest index a back-reference may reach (member start or window start) */
  Ev* ev;
  uint64_t nev, evcap;
  uint64_t end;
  int end_kind;
  int rc;                     /* D_OK, D_BAD, D_TRUNC, D_MEM; D_INPUT: stopped at the last complete unit */
  int overshoot;              /* passed stop_at without landing on it */
  /* resolution */
  uint8_t win[WIN];           /* the resolved window before the region */
  uint64_t out_off;           /* where its output goes in the batch's output */
  Tables t;
} Region;

static int reserve(Region* r, uint64_t more) {
  if (r->n + more <= r->cap) return 0;
  uint64_t c = r->cap ? r->cap : (1u << 21);
  while (c < r->n + more) c *= 2;
  uint16_t* q = (uint16_t*)realloc(r->o, c * sizeof(uint16_t));
  if (!q) return -1;
  r->o = q;
  r->cap = c;
  return 0;
}

static int add_ev(Region* r, uint64_t bit, uint32_t kind, uint32_t crc, uint64_t isize) {
  if (r->nev == r->evcap) {
    const uint64_t c = r->evcap ? 2 * r->evcap : 256;
    Ev* q = (Ev*)realloc(r->ev, c * sizeof(Ev));
    if (!q) return -1;
    r->ev = q;
    r->evcap = c;
  }
  Ev* e = &r->ev[r->nev++];
  e->bit = bit;
  e->out = r->n;
  e->kind = kind;
  e->crc = crc;
  e->isize = isize;
  return 0;
}

/* A dynamic block's code tables; *pos just after the 3 header bits.  0 ok, -1 not a valid header, -2 the
 * header runs past the input. */
static int read_dynamic_(const uint8_t* buf, uint64_t nbytes, uint64_t* pos, Tables* t, uint64_t* at);
static int read_dynamic(const uint8_t* buf, uint64_t nbytes, uint64_t* pos, Tables* t) {
  uint64_t at = *pos;
  const int rc = read_dynamic_(buf, nbytes, pos, t, &at);
  if (rc == -1 && at + 64 > nbytes * 8) return -2;      /* failed on the zeros past the end of the input */
  return rc;
}
static int read_dynamic_(const uint8_t* buf, uint64_t nbytes, uint64_t* pos, Tables* t, uint64_t* at) {
  uint64_t p = *pos;
  uint64_t v = peek_at(buf, nbytes, p);
  const uint32_t hlit = (uint32_t)(v & 31) + 257, hdist = (uint32_t)((v >> 5) & 31) + 1,
                 hclen = (uint32_t)((v >> 10) & 15) + 4;
  p += 14;
  if (hlit > 286 || hdist > 30) return -1;
  uint8_t cl[19];
  memset(cl, 0, sizeof(cl));
  v = peek_at(buf, nbytes, p);
  for (uint32_t i = 0; i < hclen; ++i) cl[kClOrder[i]] = (uint8_t)((v >> (3 * i)) & 7);
  p += 3 * hclen;
  uint32_t cltab[CLTAB];
  if (build_table(cltab, CLTAB, cl, 19, 7, 0)) return -1;
  uint8_t lens[320];
  uint32_t i = 0;
  *at = p;
  while (i < hlit + hdist) {
    *at = p;
    v = peek_at(buf, nbytes, p);
    const uint32_t e = cltab[v & 127u];
    const uint32_t l = (e >> 16) & 31u;
    if (!l) return -1;
    p += l;
    v >>= l;
    const uint32_t sym = e & 0xFFFFu;
    if (sym < 16) {
      lens[i++] = (uint8_t)sym;
    } else if (sym == 16) {
      if (i == 0) return -1;
      const uint32_t r = 3 + (uint32_t)(v & 3);
      p += 2;
      if (i + r > hlit + hdist) return -1;
      for (uint32_t k = 0; k < r; ++k, ++i) lens[i] = lens[i - 1];
    } else {
      const uint32_t r = sym == 17 ? 3 + (uint32_t)(v & 7) : 11 + (uint32_t)(v & 127);
      p += sym == 17 ? 3 : 7;
      if (i + r > hlit + hdist) return -1;
      memset(lens + i, 0, r);
      i += r;
    }
    if (p > nbytes * 8) return -2;
  }
  *at = p;
  if (!lens[256]) return -1;                            /* no end-of-block code */
  if (build_table(t->lit, LTAB, lens, (int)hlit, LBITS, 0)) return -1;
  if (build_table(t->dist, DTAB, lens + hlit, (int)hdist, DBITS, 1)) return -1;
  *pos = p;
  return 0;
}

/* A block's symbols up to and including end-of-block. */
/* Fast path: a 64-bit bit buffer refilled 8 bytes at a time (>= 56 valid bits after a refill: one
 * literal/length code, its extra bits, a distance code and its extra bits need at most 48), while at least
 * 16 input bytes remain.  Returns 1 to continue in the careful loop below, or a final D_* status. */
static int decode_fast(const uint8_t* buf, uint64_t nbytes, uint64_t* pos_io, const Tables* t, Region* r) {
  if (nbytes < 16) return 1;
  const uint8_t* ip = buf + (*pos_io >> 3);
  const uint8_t* const iend = buf + nbytes - 16;
  if (ip >= iend) return 1;
  uint64_t bb;
  uint32_t bc;
  {
    memcpy(&bb, ip, 8);
    ip += 7;
    const uint32_t sh = (uint32_t)(*pos_io & 7);
    bb >>= sh;
    bc = 56 - sh;
  }
  const uint32_t* lit = t->lit;
  const uint32_t* dst = t->dist;
  int res = 1;
  for (;;) {
    if (r->n + 600 >= r->cap && reserve(r, 1u << 20)) { res = D_MEM; break; }
    uint16_t* o = r->o;
    uint64_t n = r->n;
    const uint64_t lim = r->cap - 600;
    while (n < lim && ip < iend) {
      /* refill to >= 56 bits */
      uint64_t w;
      memcpy(&w, ip, 8);
      bb |= w << bc;
      ip += (63 - bc) >> 3;
      bc |= 56;
      uint32_t e = lit[bb & ((1u << LBITS) - 1)];
      uint32_t used;
      if (e & E_SUB) {
        e = lit[(e & 0xFFFFu) + ((bb >> LBITS) & ((1u << ((e >> 24) & 15u)) - 1))];
        used = LBITS + ((e >> 16) & 31u);
      } else {
        used = (e >> 16) & 31u;
      }
      if (!((e >> 16) & 31u)) { res = D_BAD; break; }
      bb >>= used;
      bc -= used;
      uint32_t sym = e & 0xFFFFu;
      if (sym < 256) {
        o[n++] = (uint16_t)sym;
        /* a second literal from the same refill (>= 41 bits left) */
        e = lit[bb & ((1u << LBITS) - 1)];
        if (!(e & E_SUB) && (e & 0xFFFFu) < 256 && ((e >> 16) & 31u)) {
          used = (e >> 16) & 31u;
          bb >>= used;
          bc -= used;
          o[n++] = (uint16_t)(e & 0xFFFFu);
        }
        continue;
      }
      if (sym == 256) { res = D_OK; break; }
      sym -= 257;
      if (sym >= 29) { res = D_BAD; break; }
      const uint32_t lx = kLenExtra[sym];
      const uint32_t len = kLenBase[sym] + (uint32_t)(bb & ((1u << lx) - 1));
      bb >>= lx;
      bc -= lx;
      uint32_t d = dst[bb & ((1u << DBITS) - 1)];
      if (d & E_SUB) {
        d = dst[(d & 0xFFFFu) + ((bb >> DBITS) & ((1u << ((d >> 24) & 15u)) - 1))];
        used = DBITS + ((d >> 16) & 31u);
      } else {
        used = (d >> 16) & 31u;
      }
      if (!((d >> 16) & 31u)) { res = D_BAD; break; }
      bb >>= used;
      bc -= used;
      const uint32_t ds = d & 0xFFFFu;
      if (ds >= 30) { res = D_BAD; break; }
      const uint32_t dx = kDistExtra[ds];
      const uint32_t dist = kDistBase[ds] + (uint32_t)(bb & ((1u << dx) - 1));
      bb >>= dx;
      bc -= dx;
      if (dist > n - r->floor) { res = D_BAD; break; }
      uint16_t* to = o + n;
      const uint16_t* from = to - dist;
      uint16_t* const end = to + len;
      if (dist >= 8) {                                   /* 16-byte chunks, over-copying into the slack */
        do {
          memcpy(to, from, 16);
          to += 8;
          from += 8;
        } while (to < end);
      } else if (dist == 1) {
        const uint16_t c = from[0];
        do { *to++ = c; } while (to < end);
      } else {
        do { *to++ = *from++; } while (to < end);
      }
      n += len;
    }
    r->n = n;
    if (res != 1 || ip >= iend) break;
  }
  *pos_io = (uint64_t)(ip - buf) * 8 - bc;
  return res;
}

static int decode_symbols(const uint8_t* buf, uint64_t nbytes, uint64_t* pos_io, const Tables* t, Region* r) {
  {
    const int f = decode_fast(buf, nbytes, pos_io, t, r);
    if (f != 1) return f;
  }
  uint64_t pos = *pos_io;
  const uint64_t nbits = nbytes * 8;
  const uint32_t* lit = t->lit;
  const uint32_t* dst = t->dist;
  for (;;) {
    if (r->n + 300 >= r->cap && reserve(r, 1u << 20)) return D_MEM;
    uint16_t* o = r->o;
    uint64_t n = r->n;
    const uint64_t lim = r->cap - 300;
    int res = 1;
    while (n < lim) {
      uint64_t v = peek_at(buf, nbytes, pos);
      uint32_t e = lit[v & ((1u << LBITS) - 1)];
      uint32_t used;
      if (e & E_SUB) {
        const uint32_t sb = (e >> 24) & 15u;
        e = lit[(e & 0xFFFFu) + ((v >> LBITS) & ((1u << sb) - 1))];
        used = LBITS + ((e >> 16) & 31u);
      } else {
        used = (e >> 16) & 31u;
      }
      if (!((e >> 16) & 31u)) { res = D_BAD; break; }
      pos += used;
      v >>= used;
      const uint32_t sym = e & 0xFFFFu;
      if (sym < 256) {
        o[n++] = (uint16_t)sym;
        if (pos > nbits) { res = D_INPUT; break; }
        continue;
      }
      if (sym == 256) {
        res = pos > nbits ? D_INPUT : D_OK;
        break;
      }
      const uint32_t ls = sym - 257;
      if (ls >= 29) { res = D_BAD; break; }
      const uint32_t lx = kLenExtra[ls];
      const uint32_t len = kLenBase[ls] + (uint32_t)(v & ((1u << lx) - 1));
      pos += lx;
      v >>= lx;
      uint32_t d = dst[v & ((1u << DBITS) - 1)];
      if (d & E_SUB) {
        const uint32_t sb = (d >> 24) & 15u;
        d = dst[(d & 0xFFFFu) + ((v >> DBITS) & ((1u << sb) - 1))];
        used = DBITS + ((d >> 16) & 31u);
      } else {
        used = (d >> 16) & 31u;
      }
      if (!((d >> 16) & 31u)) { res = D_BAD; break; }
      pos += used;
      v >>= used;
      const uint32_t ds = d & 0xFFFFu;
      if (ds >= 30) { res = D_BAD; break; }
      const uint32_t dx = kDistExtra[ds];
      const uint32_t dist = kDistBase[ds] + (uint32_t)(v & ((1u << dx) - 1));
      pos += dx;
      if (pos > nbits) { res = D_INPUT; break; }
      if (dist > n - r->floor) { res = D_BAD; break; }
      uint16_t* to = o + n;
      const uint16_t* from = to - dist;
      if (dist >= len) {
        memcpy(to, from, (size_t)len * 2);
      } else {
        for (uint32_t k = 0; k < len; ++k) to[k] = from[k];
      }
      n += len;
    }
    r->n = n;
    if (res != 1) {
      /* an invalid code read from the zeros past the end of the input: the input ended */
      if (res == D_BAD && pos + 64 > nbits) res = D_INPUT;
      *pos_io = pos;
      return res;
    }
  }
}

/* gzip member header at byte p: 0 and *hend = the first byte after it, -1 invalid, -2 incomplete. */
static int parse_header(const uint8_t* b, uint64_t n, uint64_t p, uint64_t* hend) {
  if (n - p < 10) return -2;
  if (b[p] != 0x1f || b[p + 1] != 0x8b || b[p + 2] != 8) return -1;
  const uint8_t flg = b[p + 3];
  if (flg & 0xE0) return -1;
  uint64_t q = p + 10;
  if (flg & 4) {
    if (n - q < 2) return -2;
    const uint64_t xlen = (uint64_t)b[q] | ((uint64_t)b[q + 1] << 8);
    q += 2 + xlen;
    if (q > n) return -2;
  }
  for (int f = 8; f <= 16; f <<= 1) {
    if (flg & f) {
      while (q < n && b[q]) ++q;
      if (q >= n) return -2;
      ++q;
    }
  }
  if (flg & 2) q += 2;
  if (q > n) return -2;
  *hend = q;
  return 0;
}

/* Decode a region: from r->start until a block start == stop_at (or past it), the end of the input
 * (D_INPUT, rolled back to the last complete unit; with `final`, a truncation error) or the end of the
 * stream (K_END, final only). */
static void decode_region(Region* r, const uint8_t* buf, uint64_t nbytes, int final) {
  pthread_once(&g_fixed_once, fixed_init);
  uint64_t pos = r->start;
  int kind = r->start_kind;
  r->n = WIN;
  r->nev = 0;
  r->floor = r->floor0;
  r->overshoot = 0;
  r->rc = D_OK;
  for (;;) {
    if (kind == K_HEADER) {
      uint64_t p = pos >> 3;
      while (p < nbytes && buf[p] == 0) ++p;            /* zero padding after a member (like gzip -d) */
      if (p == nbytes) {
        r->end = pos;
        r->end_kind = final ? K_END : K_HEADER;
        r->rc = final ? D_OK : D_INPUT;
        if (final) r->end = p * 8;
        return;
      }
      uint64_t hend = 0;
      const int h = parse_header(buf, nbytes, p, &hend);
      if (h == -2) {
        r->end = p * 8;
        r->end_kind = K_HEADER;
        r->rc = final ? D_TRUNC : D_INPUT;
        return;
      }
      if (h) { r->rc = D_BAD; r->end = p * 8; r->end_kind = K_HEADER; return; }
      if (add_ev(r, p * 8, EV_MSTART, 0, 0)) { r->rc = D_MEM; return; }
      r->floor = r->n;                                  /* no reference reaches before a member start */
      pos = hend * 8;
      kind = K_BLOCK;
      continue;
    }
    if (pos == r->stop_at || (r->stop_at == NONE && pos >= r->stop_after)) {
      r->end = pos;
      r->end_kind = K_BLOCK;
      return;
    }
    if (r->stop_at != NONE && pos > r->stop_at) { r->overshoot = 1; r->end = pos; r->end_kind = K_BLOCK; return; }
    const uint64_t bstart = pos, ostart = r->n, evmark = r->nev;
    if (add_ev(r, pos, EV_BLOCK, 0, 0)) { r->rc = D_MEM; return; }
    const uint64_t hv = peek_at(buf, nbytes, pos);
    const uint32_t bfinal = (uint32_t)(hv & 1), btype = (uint32_t)((hv >> 1) & 3);
    pos += 3;
    int res = D_OK;
    if (btype == 0) {
      uint64_t p = (pos + 7) >> 3;
      if (p + 4 > nbytes) {
        res = D_INPUT;
      } else {
        const uint32_t len = (uint32_t)buf[p] | ((uint32_t)buf[p + 1] << 8);
        const uint32_t nlen = (uint32_t)buf[p + 2] | ((uint32_t)buf[p + 3] << 8);
        if ((len ^ 0xFFFFu) != nlen) {
          res = D_BAD;
        } else if (p + 4 + len > nbytes) {
          res = D_INPUT;
        } else if (reserve(r, len)) {
          res = D_MEM;
        } else {
          for (uint32_t k = 0; k < len; ++k) r->o[r->n + k] = buf[p + 4 + k];
          r->n += len;
          pos = (p + 4 + len) * 8;
        }
      }
    } else if (btype == 1) {
      res = decode_symbols(buf, nbytes, &pos, &g_fixed, r);
    } else if (btype == 2) {
      const int h = read_dynamic(buf, nbytes, &pos, &r->t);
      res = h == -2 ? D_INPUT : h ? D_BAD : decode_symbols(buf, nbytes, &pos, &r->t, r);
    } else {
      res = D_BAD;
    }
    if (res == D_OK && bfinal) {                        /* member end: byte-aligned 8-byte trailer */
      const uint64_t p = (pos + 7) >> 3;
      if (p + 8 > nbytes) {
        res = D_INPUT;
      } else {
        const uint32_t crc = (uint32_t)buf[p] | ((uint32_t)buf[p + 1] << 8) | ((uint32_t)buf[p + 2] << 16) |
                             ((uint32_t)buf[p + 3] << 24);
        const uint64_t isz = (uint64_t)buf[p + 4] | ((uint64_t)buf[p + 5] << 8) | ((uint64_t)buf[p + 6] << 16) |
                             ((uint64_t)buf[p + 7] << 24);
        if (add_ev(r, (p + 8) * 8, EV_MEND, crc, isz)) { r->rc = D_MEM; return; }
        pos = (p + 8) * 8;
        kind = K_HEADER;
      }
    }
    if (res == D_INPUT) {                               /* roll the unfinished block back */
      r->n = ostart;
      r->nev = evmark;
      r->end = bstart;
      r->end_kind = K_BLOCK;
      r->rc = final ? D_TRUNC : D_INPUT;
      return;
    }
    if (res != D_OK) {
      r->n = ostart;
      r->nev = evmark;
      r->end = bstart;
      r->end_kind = K_BLOCK;
      r->rc = res;
      return;
    }
  }
}

/* First position in [from, to) where a non-final dynamic block starts and decodes to its end (NONE if none). */
static uint64_t find_block(Region* r, const uint8_t* buf, uint64_t nbytes, uint64_t from, uint64_t to) {
  pthread_once(&g_fixed_once, fixed_init);
  for (uint64_t pos = from; pos < to; ++pos) {
    const uint64_t v = peek_at(buf, nbytes, pos);
    if ((v & 7) != 4) continue;                         /* BFINAL 0, BTYPE 2 */
    if (((v >> 3) & 31) > 29 || ((v >> 8) & 31) > 29) continue;
    const uint32_t hclen = (uint32_t)((v >> 13) & 15) + 4;
    const uint64_t w = peek_at(buf, nbytes, pos + 17);
    int left = 128;                                     /* Kraft sum of the code-length code, x 128 */
    for (uint32_t i = 0; i < hclen; ++i) {
      const uint32_t l = (uint32_t)((w >> (3 * i)) & 7);
      if (l) left -= 128 >> l;
    }
    if (left != 0) continue;
    uint64_t p = pos + 3;
    if (read_dynamic(buf, nbytes, &p, &r->t)) continue;
    r->n = WIN;
    r->floor = 0;
    if (decode_symbols(buf, nbytes, &p, &r->t, r) == D_OK) return pos;
  }
  return NONE;
}

/* One complete gzip member (header to trailer, nothing after it but zero padding) into out[0, out_len)
 * exactly, CRC-32 and ISIZE checked; the BGZF member-parallel path.  *scratch: a decoder state this
 * thread reuses (NULL at first; free with dpgz__member_free). */
int dpgz__member(const uint8_t* gz, uint64_t len, uint8_t* out, uint64_t out_len, void** scratch) {
  Region* r = (Region*)*scratch;
  if (!r) {
    r = (Region*)calloc(1, sizeof(Region));
    if (!r) return DPGZ_ERR_MEMORY;
    *scratch = r;
  }
  r->start = 0;
  r->start_kind = K_HEADER;
  r->stop_at = NONE;
  r->stop_after = NONE;
  r->floor0 = WIN;
  r->n = 0;
  if (reserve(r, WIN + out_len + 1024)) return DPGZ_ERR_MEMORY;
  decode_region(r, gz, len, 1);
  if (r->rc == D_MEM) return DPGZ_ERR_MEMORY;
  if (r->rc == D_TRUNC) return DPGZ_ERR_TRUNCATED;
  if (r->rc != D_OK || r->end_kind != K_END) return DPGZ_ERR_ZLIB;
  const uint64_t m = r->n - WIN;
  uint32_t crc = 0, nmend = 0;
  uint64_t isize = 0;
  for (uint64_t e = 0; e < r->nev; ++e)
    if (r->ev[e].kind == EV_MEND) { crc = r->ev[e].crc; isize = r->ev[e].isize; ++nmend; }
  if (nmend != 1 || m != out_len || (m & 0xFFFFFFFFull) != isize) return DPGZ_ERR_ZLIB;
  const uint16_t* o = r->o + WIN;
  for (uint64_t i = 0; i < m; ++i) out[i] = (uint8_t)o[i];
  if (crc32_fast(0u, out, m) != crc) return DPGZ_ERR_ZLIB;
  return DPGZ_OK;
}

void dpgz__member_free(void* scratch) {
  Region* r = (Region*)scratch;
  if (!r) return;
  free(r->o);
  free(r->ev);
  free(r);
}


/* ------------------------------------------------------------------------------------------ the engine */
/* ---- a parallel-for over a pool of worker threads that live as long as the engine (one batch runs 2-4
 * parallel loops; creating and joining 15 threads per loop cost ~1 ms per batch) */
typedef struct {
  void (*fn)(void*, int);
  void* arg;
  int n;
  int next;
} PFor;
static void pfor_worker(PFor* p) {
  for (;;) {
    const int i = __atomic_fetch_add(&p->next, 1, __ATOMIC_RELAXED);
    if (i >= p->n) break;
    p->fn(p->arg, i);
  }
}
struct Pool;
typedef struct {
  struct Pool* p;
  int id;
} PoolWorker;
typedef struct Pool {
  pthread_t th[256];
  PoolWorker w[256];
  int n;                      /* workers (the calling thread is one more) */
  pthread_mutex_t m;
  pthread_cond_t go, done;
  uint64_t gen;
  int quit, active;
  int limit;                  /* workers taking part in the current loop */
  PFor* job;
} Pool;
static void* pool_main(void* a) {
  PoolWorker* me = (PoolWorker*)a;
  Pool* p = me->p;
  uint64_t seen = 0;
  pthread_mutex_lock(&p->m);
  for (;;) {
    while (p->gen == seen && !p->quit) pthread_cond_wait(&p->go, &p->m);
    if (p->quit) break;
    seen = p->gen;
    PFor* j = p->job;
    const int take = me->id < p->limit;
    pthread_mutex_unlock(&p->m);
    if (take) pfor_worker(j);
    pthread_mutex_lock(&p->m);
    if (--p->active == 0) pthread_cond_signal(&p->done);
  }
  pthread_mutex_unlock(&p->m);
  return NULL;
}
static int pool_init(Pool* p, int workers) {
  memset(p, 0, sizeof(*p));
  pthread_mutex_init(&p->m, NULL);
  pthread_cond_init(&p->go, NULL);
  pthread_cond_init(&p->done, NULL);
  for (int t = 0; t < workers && t < 256; ++t) {
    p->w[t].p = p;
    p->w[t].id = t;
    if (pthread_create(&p->th[t], NULL, pool_main, &p->w[t]) != 0) break;
    p->n++;
  }
  return 0;
}
static void pool_free(Pool* p) {
  pthread_mutex_lock(&p->m);
  p->quit = 1;
  pthread_cond_broadcast(&p->go);
  pthread_mutex_unlock(&p->m);
  for (int t = 0; t < p->n; ++t) pthread_join(p->th[t], NULL);
  pthread_cond_destroy(&p->go);
  pthread_cond_destroy(&p->done);
  pthread_mutex_destroy(&p->m);
}
/* fn(arg, i) for i in [0, n) on the calling thread and up to threads - 1 of the pool's workers */
static void pool_for_n(Pool* p, int threads, int n, void (*fn)(void*, int), void* arg) {
  PFor j = {fn, arg, n, 0};
  if (p->n == 0 || n <= 1 || threads <= 1) {
    pfor_worker(&j);
    return;
  }
  pthread_mutex_lock(&p->m);
  p->job = &j;
  p->limit = threads - 1;
  p->active = p->n;
  p->gen++;
  pthread_cond_broadcast(&p->go);
  pthread_mutex_unlock(&p->m);
  pfor_worker(&j);
  pthread_mutex_lock(&p->m);
  while (p->active) pthread_cond_wait(&p->done, &p->m);
  pthread_mutex_unlock(&p->m);
}
static void pool_for(Pool* p, int n, void (*fn)(void*, int), void* arg) { pool_for_n(p, p->n + 1, n, fn, arg); }

/* The BGZF member-parallel path (dpgz.c) runs on one process-wide pool, created at the first call with
 * that call's thread count and kept (no thread creation per batch of members); calls are serialized.  Each
 * thread keeps its member decoder state across calls (pthread key, freed at thread exit). */
static Pool g_pool;
static int g_pool_ready;
static pthread_mutex_t g_pool_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_key_t g_scratch_key;
static pthread_once_t g_scratch_once = PTHREAD_ONCE_INIT;
static void scratch_key_init(void) { pthread_key_create(&g_scratch_key, dpgz__member_free); }
void* dpgz__scratch_get(void) {
  pthread_once(&g_scratch_once, scratch_key_init);
  return pthread_getspecific(g_scratch_key);
}
void dpgz__scratch_put(void* scratch) {
  pthread_once(&g_scratch_once, scratch_key_init);
  pthread_setspecific(g_scratch_key, scratch);
}
static void pool_after_fork_child(void) {   /* the workers do not exist in a forked child: start over */
  pthread_mutex_init(&g_pool_mu, NULL);
  g_pool_ready = 0;
}
void dpgz__global_for(int threads, int n, void (*fn)(void*, int), void* arg) {
  if (threads > 256) threads = 256;
  pthread_mutex_lock(&g_pool_mu);
  if (g_pool_ready && g_pool.n < threads - 1) {         /* more threads than the pool has: regrow it */
    pool_free(&g_pool);
    g_pool_ready = 0;
  }
  if (!g_pool_ready) {
    static int atfork_done;
    if (!atfork_done) {
      pthread_atfork(NULL, NULL, pool_after_fork_child);
      atfork_done = 1;
    }
    pool_init(&g_pool, threads - 1);
    g_pool_ready = 1;
  }
  pool_for_n(&g_pool, threads, n, fn, arg);
  pthread_mutex_unlock(&g_pool_mu);
}

struct dpgz_par {
  uint64_t span;
  int threads;
  uint8_t* cin;               /* pending compressed bytes; cin[0] is stream byte cbase */
  uint64_t clen, ccap, cbase;
  uint64_t pos;               /* next unit: bit position in cin */
  int kind;
  uint8_t win[WIN];           /* the current member's last (up to) WIN inflated bytes before pos */
  uint32_t wl;
  uint64_t out_total;         /* inflated bytes produced */
  uint64_t members;
  uint32_t crc;               /* running CRC-32 / length of the current member */
  uint64_t msize;
  uint64_t mstart_out;        /* output offset where the current member starts */
  uint64_t last;              /* output offset of the last access point */
  int32_t prev;
  uint8_t* out;               /* resolved output not yet read: [ohead, olen) */
  uint64_t ohead, olen, ocap;
  dpgz_point_ex* pts;         /* points not yet taken */
  uint64_t npts, pcap;
  uint8_t* wins;
  uint64_t nwin, wcap;
  int failed;
  Region* regs;
  int nregs;
  uint64_t batches, rejected;
  uint64_t region_min;
  Pool pool;                  /* threads - 1 workers */
  uint64_t ns[5];             /* time per phase: find, decode, windows, resolve, in-order bookkeeping */
};

int dpgz_par_new(uint64_t span, int threads, dpgz_par** out) {
  if (!out) return DPGZ_ERR_INVALID;
  dpgz_par* s = (dpgz_par*)calloc(1, sizeof(dpgz_par));
  if (!s) return DPGZ_ERR_MEMORY;
  s->span = span ? span : (1u << 20);
  s->threads = threads > 0 ? (threads > 256 ? 256 : threads) : 1;
  s->kind = K_HEADER;
  s->region_min = REGION_MIN;
  s->prev = -1;
  s->crc = (uint32_t)crc32(0L, Z_NULL, 0);
  s->nregs = 2 * s->threads;                          /* regions per batch: two per thread (dynamic balance) */
  s->regs = (Region*)calloc((size_t)s->nregs, sizeof(Region));
  if (!s->regs) { free(s); return DPGZ_ERR_MEMORY; }
  pool_init(&s->pool, s->threads - 1);
  *out = s;
  return DPGZ_OK;
}

void dpgz_par_free(dpgz_par* s) {
  if (!s) return;
  pool_free(&s->pool);
  for (int i = 0; i < s->nregs; ++i) {
    free(s->regs[i].o);
    free(s->regs[i].ev);
  }
  free(s->regs);
  free(s->cin);
  free(s->out);
  free(s->pts);
  free(s->wins);
  free(s);
}

typedef struct {
  dpgz_par* s;
  int final;
  uint64_t nbytes;
  uint64_t* bound;            /* nominal region starts (bits), nreg + 1 */
  uint64_t* found;            /* found starts */
  int* idx;                   /* region slot of each kept start */
  int nkeep;
  int nreg;
  uint64_t stop_last;         /* the last region's stop_after (NONE: the batch holds the rest of the input) */
  uint8_t* dst;               /* the batch's resolved output */
  uint32_t* seg_crc;          /* per region: CRC of its output up to its first member end, then per member */
  uint64_t* seg_len;
  uint64_t* seg_off;          /* first segment of each region in seg_* */
} Batch;

static void job_find_decode(void* a, int i) {
  Batch* b = (Batch*)a;
  dpgz_par* s = b->s;
  Region* r = &s->regs[i];
  r->n = 0;                                             /* the buffer is reused: only the window is kept */
  if (reserve(r, WIN + s->region_min * 5 / 2 + (1u << 16))) { r->rc = D_MEM; return; }
  if (i > 0) {
    b->found[i] = find_block(r, s->cin, b->nbytes, b->bound[i], b->bound[i + 1]);
    if (b->found[i] == NONE) { r->rc = D_OK; return; }
  }
  r->start = i == 0 ? s->pos : b->found[i];
  r->start_kind = i == 0 ? s->kind : K_BLOCK;
  r->stop_at = NONE;
  r->stop_after = i + 1 < b->nreg ? b->bound[i + 1] : b->stop_last;
  if (i == 0) {                                         /* the known window, right-aligned */
    for (uint32_t j = 0; j < WIN; ++j) r->o[j] = j >= WIN - s->wl ? s->win[j - (WIN - s->wl)] : (uint16_t)(256 + j);
    r->floor0 = WIN - s->wl;
  } else {
    for (uint32_t j = 0; j < WIN; ++j) r->o[j] = (uint16_t)(256 + j);
    r->floor0 = 0;
  }
  decode_region(r, s->cin, b->nbytes, b->final && i == b->nreg - 1);
}

static void job_resolve(void* a, int k) {
  Batch* b = (Batch*)a;
  Region* r = &b->s->regs[b->idx[k]];
  uint8_t* d = b->dst + r->out_off;
  const uint16_t* o = r->o + WIN;
  const uint64_t m = r->n - WIN;
  uint64_t i = 0;
  while (i < m) {                                       /* 32 symbols at a time while no marker is among them */
    if (i + 32 <= m) {
      uint16_t any = 0;
      for (int k = 0; k < 32; ++k) any |= o[i + k];
      if (!(any & 0xFF00u)) {
        for (int k = 0; k < 32; ++k) d[i + k] = (uint8_t)o[i + k];
        i += 32;
        continue;
      }
    }
    const uint64_t e = i + 32 < m ? i + 32 : m;
    for (; i < e; ++i) {
      const uint16_t v = o[i];
      d[i] = v < 256 ? (uint8_t)v : r->win[v - 256];
    }
  }
  /* CRC segments, split at member ends and starts (a member's CRC covers its own bytes only) */
  uint64_t si = b->seg_off[k], from = 0;
  for (uint64_t e = 0; e < r->nev; ++e) {
    if (r->ev[e].kind == EV_BLOCK) continue;
    const uint64_t at = r->ev[e].out - WIN;
    b->seg_crc[si] = crc32_fast(0u, d + from, at - from);
    b->seg_len[si] = at - from;
    ++si;
    from = at;
  }
  b->seg_crc[si] = crc32_fast(0u, d + from, m - from);
  b->seg_len[si] = m - from;
}

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

/* Queue an access point at output offset `out` with its window (the current member's last <= WIN bytes
 * before it) and the byte before it.  hist: contiguous inflated bytes, hist[0] at output offset hist_base,
 * covering at least WIN bytes before `out` (or everything since the stream start). */
static int add_point(dpgz_par* s, uint64_t in_byte, uint32_t bits, uint64_t out, uint32_t member,
                     const uint8_t* hist, uint64_t hist_base) {
  if (grow((void**)&s->pts, &s->pcap, s->npts + 1, sizeof(dpgz_point_ex))) return -1;
  dpgz_point_ex* p = &s->pts[s->npts++];
  p->in_byte = in_byte;
  p->out_byte = out;
  p->bits = bits;
  p->member_start = member;
  p->prev_byte = out > hist_base ? (int32_t)hist[out - 1 - hist_base] : (out == 0 ? -1 : s->prev);
  p->window_len = 0;
  if (!member) {
    uint64_t w0 = out > WIN ? out - WIN : 0;
    if (w0 < s->mstart_out) w0 = s->mstart_out;
    if (w0 < hist_base) return -1;                       /* the caller keeps >= WIN bytes of history */
    const uint64_t wl = out - w0;
    if (grow((void**)&s->wins, &s->wcap, s->nwin + wl, 1)) return -1;
    memcpy(s->wins + s->nwin, hist + (w0 - hist_base), wl);
    s->nwin += wl;
    p->window_len = (uint32_t)wl;
  }
  s->last = out;
  return 0;
}

/* One batch over the pending compressed bytes.  Returns a DPGZ status; *progress = 1 if it moved. */
static uint64_t now_ns(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
static int par_batch(dpgz_par* s, int final, int* progress) {
  *progress = 0;
  uint64_t t0 = now_ns(), t1;
  if (s->kind == K_END) return DPGZ_OK;
  const uint64_t nbytes = s->clen;
  const uint64_t b0 = s->pos >> 3;
  /* at most two batches' worth of regions at a time (bounded memory whatever the caller feeds); the last
   * region then stops at the first block start past the batch and the rest waits for the next batch */
  const uint64_t cap_bytes = 2ull * (uint64_t)s->nregs * s->region_min;
  const int whole = nbytes - b0 <= cap_bytes;
  const uint64_t avail = whole ? nbytes - b0 : cap_bytes;
  if (!whole) final = 0;
  int nreg = (int)(avail / s->region_min);
  if (nreg > s->nregs) nreg = s->nregs;
  if (nreg < 1) nreg = 1;
  uint64_t bound[2 * 256 + 1], found[2 * 256 + 1];
  int idx[2 * 256 + 1];
  for (int i = 0; i <= nreg; ++i) bound[i] = (b0 + avail * (uint64_t)i / (uint64_t)nreg) * 8;
  bound[0] = s->pos;
  found[0] = s->pos;
  Batch B;
  memset(&B, 0, sizeof(B));
  B.s = s;
  B.final = final;
  B.nbytes = nbytes;
  B.bound = bound;
  B.found = found;
  B.idx = idx;
  B.nreg = nreg;
  B.stop_last = whole ? NONE : (b0 + avail) * 8;
  /* every region: find its start (a block start in its nominal range; region 0 starts at the known position),
   * then decode to the first block start at or past the next region's nominal start -- which is that
   * region's found start when it is a true one.  Regions outnumber the threads (dynamic balance). */
  pool_for(&s->pool, nreg, job_find_decode, &B);
  t1 = now_ns(); s->ns[1] += t1 - t0; t0 = t1;
  /* keep regions in order while each starts exactly where the previous kept one stopped (a region without
   * a block start in its range is skipped: the previous one decodes through it) */
  int nkeep = 0;
  for (int i = 0; i < nreg; ++i) {
    Region* r = &s->regs[i];
    if (i > 0) {
      if (found[i] == NONE) continue;
      Region* q = &s->regs[idx[nkeep - 1]];
      if (q->rc != D_OK || q->end != r->start) {
        if (q->rc == D_OK) s->rejected++;
        break;
      }
    }
    if (r->rc == D_MEM) return DPGZ_ERR_MEMORY;
    if (r->rc == D_BAD) return DPGZ_ERR_ZLIB;           /* its start is a true boundary: corrupt data */
    if (r->rc == D_TRUNC) return DPGZ_ERR_TRUNCATED;
    idx[nkeep++] = i;
    if (r->rc == D_INPUT) break;
  }
  Region* lastr = &s->regs[idx[nkeep - 1]];
  uint64_t total = 0;
  for (int k = 0; k < nkeep; ++k) {
    Region* r = &s->regs[idx[k]];
    r->out_off = total;
    total += r->n - WIN;
  }
  if (total == 0 && lastr->end == s->pos && lastr->end_kind == s->kind && lastr->rc == D_INPUT) return DPGZ_OK;
  /* windows, in order: region 0's is the known one; region k's = the resolved last WIN entries of k-1 */
  {
    Region* r0 = &s->regs[idx[0]];
    memset(r0->win, 0, WIN);
    memcpy(r0->win + (WIN - s->wl), s->win, s->wl);
    for (int k = 1; k < nkeep; ++k) {
      Region* q = &s->regs[idx[k - 1]];
      Region* r = &s->regs[idx[k]];
      const uint16_t* t = q->o + q->n - WIN;
      for (uint32_t j = 0; j < WIN; ++j) r->win[j] = t[j] < 256 ? (uint8_t)t[j] : q->win[t[j] - 256];
    }
  }
  /* output space: [ohead, olen) unread + total; keep >= WIN bytes before the batch for the points' windows */
  if (s->ohead > 2 * WIN && s->ohead > s->olen / 2) {
    const uint64_t drop = s->ohead - WIN;
    memmove(s->out, s->out + drop, s->olen - drop);
    s->olen -= drop;
    s->ohead -= drop;
  }
  if (grow((void**)&s->out, &s->ocap, s->olen + total + 1, 1)) return DPGZ_ERR_MEMORY;
  uint64_t nseg = 0;
  uint64_t seg_off[257];
  for (int k = 0; k < nkeep; ++k) {
    Region* r = &s->regs[idx[k]];
    seg_off[k] = nseg;
    for (uint64_t e = 0; e < r->nev; ++e) nseg += r->ev[e].kind != EV_BLOCK;
    ++nseg;
  }
  uint32_t* seg_crc = (uint32_t*)malloc(nseg * sizeof(uint32_t));
  uint64_t* seg_len = (uint64_t*)malloc(nseg * sizeof(uint64_t));
  if (!seg_crc || !seg_len) { free(seg_crc); free(seg_len); return DPGZ_ERR_MEMORY; }
  B.dst = s->out + s->olen;
  B.seg_crc = seg_crc;
  B.seg_len = seg_len;
  B.seg_off = seg_off;
  B.nkeep = nkeep;
  t1 = now_ns(); s->ns[2] += t1 - t0; t0 = t1;
  pool_for(&s->pool, nkeep, job_resolve, &B);
  t1 = now_ns(); s->ns[3] += t1 - t0; t0 = t1;
  /* in order: CRC / ISIZE per member, access points with their windows */
  int rc = DPGZ_OK;
  const uint8_t* hist = s->out;                         /* output offset of hist[0]: */
  const uint64_t hist_base = s->out_total - s->olen;
  for (int k = 0; k < nkeep && rc == DPGZ_OK; ++k) {
    Region* r = &s->regs[idx[k]];
    uint64_t si = seg_off[k];
    const uint64_t rbase = s->out_total + r->out_off;   /* output offset of the region's first byte */
    for (uint64_t e = 0; e < r->nev && rc == DPGZ_OK; ++e) {
      const Ev* ev = &r->ev[e];
      const uint64_t at = rbase + (ev->out - WIN);
      if (ev->kind == EV_BLOCK) {
        if (at - s->last >= s->span && at > s->mstart_out) {
          const uint64_t in_byte = (ev->bit + 7) >> 3;
          if (add_point(s, s->cbase + in_byte, (uint32_t)(in_byte * 8 - ev->bit), at, 0, hist, hist_base))
            rc = DPGZ_ERR_MEMORY;
        }
        continue;
      }
      s->crc = (uint32_t)crc32_combine(s->crc, seg_crc[si], (z_off_t)seg_len[si]);
      s->msize += seg_len[si];
      ++si;
      if (ev->kind == EV_MEND) {
        if (s->crc != ev->crc || (s->msize & 0xFFFFFFFFull) != ev->isize) rc = DPGZ_ERR_ZLIB;
      } else {                                          /* EV_MSTART */
        s->crc = (uint32_t)crc32(0L, Z_NULL, 0);
        s->msize = 0;
        s->mstart_out = at;
        s->members++;
        if (add_point(s, s->cbase + (ev->bit >> 3), 0, at, 1, hist, hist_base)) rc = DPGZ_ERR_MEMORY;
      }
    }
    s->crc = (uint32_t)crc32_combine(s->crc, seg_crc[si], (z_off_t)seg_len[si]);
    s->msize += seg_len[si];
  }
  free(seg_crc);
  free(seg_len);
  if (rc != DPGZ_OK) return rc;
  s->olen += total;
  s->out_total += total;
  if (s->olen) s->prev = s->out[s->olen - 1];
  /* the window for the next batch: the current member's last WIN bytes */
  s->kind = lastr->end_kind;
  if (s->kind == K_BLOCK) {
    uint64_t w0 = s->out_total > WIN ? s->out_total - WIN : 0;
    if (w0 < s->mstart_out) w0 = s->mstart_out;
    if (w0 < hist_base) return DPGZ_ERR_INVALID;         /* >= WIN bytes of history are always kept */
    const uint64_t wl = s->out_total - w0;
    memcpy(s->win, s->out + (w0 - hist_base), wl);
    s->wl = (uint32_t)wl;
  } else {
    s->wl = 0;
  }
  /* drop the consumed compressed bytes */
  const uint64_t endb = lastr->end >> 3;
  memmove(s->cin, s->cin + endb, s->clen - endb);
  s->clen -= endb;
  s->cbase += endb;
  s->pos = lastr->end - endb * 8;
  s->batches++;
  *progress = 1;
  s->ns[4] += now_ns() - t0;
  return DPGZ_OK;
}

typedef struct {
  uint8_t* dst;
  const uint8_t* src;
  uint64_t n;
} CopyJob;
#define COPY_PART (1u << 20)
static void job_copy(void* a, int i) {
  CopyJob* c = (CopyJob*)a;
  const uint64_t o = (uint64_t)i * COPY_PART;
  memcpy(c->dst + o, c->src + o, c->n - o < COPY_PART ? c->n - o : COPY_PART);
}

int dpgz_par_set_region(dpgz_par* s, uint64_t bytes) {
  if (!s || bytes < 64) return DPGZ_ERR_INVALID;
  s->region_min = bytes;
  return DPGZ_OK;
}

int dpgz_par_feed(dpgz_par* s, const uint8_t* in, uint64_t in_len, int in_final) {
  if (!s || (!in && in_len)) return DPGZ_ERR_INVALID;
  if (s->failed) return s->failed;
  if (grow((void**)&s->cin, &s->ccap, s->clen + in_len + 8, 1)) return s->failed = DPGZ_ERR_MEMORY;
  if (in_len >= 4 * COPY_PART && s->threads > 1) {
    CopyJob c = {s->cin + s->clen, in, in_len};
    pool_for(&s->pool, (int)((in_len + COPY_PART - 1) / COPY_PART), job_copy, &c);
  } else if (in_len) {
    memcpy(s->cin + s->clen, in, in_len);
  }
  s->clen += in_len;
  const uint64_t want = (uint64_t)s->nregs * s->region_min;
  for (;;) {
    if (s->kind == K_END) break;
    const uint64_t avail = s->clen - (s->pos >> 3);
    if (!in_final && avail < want) break;
    int progress = 0;
    const int rc = par_batch(s, in_final, &progress);
    if (rc) return s->failed = rc;
    if (!progress) {
      if (in_final) return s->failed = DPGZ_ERR_TRUNCATED;
      break;
    }
  }
  return DPGZ_OK;
}

int dpgz_par_read(dpgz_par* s, uint8_t* out, uint64_t cap, uint64_t* n) {
  if (!s || !n || (!out && cap)) return DPGZ_ERR_INVALID;
  const uint64_t k = s->olen - s->ohead < cap ? s->olen - s->ohead : cap;
  if (k >= 4 * COPY_PART && s->threads > 1) {         /* into pinned pieces: one copy, on all threads */
    CopyJob c = {out, s->out + s->ohead, k};
    pool_for(&s->pool, (int)((k + COPY_PART - 1) / COPY_PART), job_copy, &c);
  } else if (k) {
    memcpy(out, s->out + s->ohead, k);
  }
  s->ohead += k;
  *n = k;
  return DPGZ_OK;
}

int dpgz_par_take(dpgz_par* s, uint64_t out_limit, dpgz_point_ex* pts, uint64_t max_pts, uint8_t* windows,
                  uint64_t win_cap, uint64_t* n_pts, uint64_t* n_win) {
  if (!s || !n_pts || !n_win) return DPGZ_ERR_INVALID;
  uint64_t n = 0, w = 0;
  while (n < s->npts && n < max_pts && s->pts[n].out_byte <= out_limit && w + s->pts[n].window_len <= win_cap) {
    w += s->pts[n].window_len;
    ++n;
  }
  if (n && (!pts || (w && !windows))) return DPGZ_ERR_INVALID;
  memcpy(pts, s->pts, n * sizeof(dpgz_point_ex));
  memcpy(windows, s->wins, w);
  memmove(s->pts, s->pts + n, (s->npts - n) * sizeof(dpgz_point_ex));
  memmove(s->wins, s->wins + w, s->nwin - w);
  s->npts -= n;
  s->nwin -= w;
  *n_pts = n;
  *n_win = w;
  return DPGZ_OK;
}

int dpgz_par_state(dpgz_par* s, uint64_t* stats) {
  if (!s || !stats) return DPGZ_ERR_INVALID;
  stats[0] = s->cbase + (s->pos >> 3);        /* compressed bytes fully consumed */
  stats[1] = s->out_total;                    /* inflated bytes produced */
  stats[2] = s->members;
  stats[3] = s->olen - s->ohead;              /* inflated bytes not read yet */
  stats[4] = s->npts;
  stats[5] = s->nwin;
  stats[6] = s->kind == K_END;                /* the stream ended */
  stats[7] = s->batches;
  stats[8] = s->rejected;                     /* region starts dropped (not a block boundary) */
  for (int i = 0; i < 5; ++i) stats[9 + i] = s->ns[i];   /* ns in find, decode, windows, resolve, bookkeeping */
  return DPGZ_OK;
}
