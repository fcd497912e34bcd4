/*
 * dpref.c — CPU ORACLE in plain C (test infrastructure only; never linked into the product).
 *
 * A byte-at-a-time restatement of the reference's FASTA header index and of a delimiter offset index,
 * fast enough (memchr-driven) to check the GPU kernels at BASELINE sizes (GiBs) and to time a scalar
 * CPU baseline.  Pinned by tests/test_oracle.py against the golden vectors the reference produced.
 *
 * dpref_fasta follows dataplug/formats/genomics/fasta.py:24-63 per chunk [c0, c1) of the reference chunk
 * plan (preprocessing/preprocess.py:38, handler.py:36-38), in the equivalent byte-state form of
 * re.finditer(rb">.+(\n)?"): scanning p upwards with seen = false, '\n' clears seen; a
 * '>' at p with !seen, p+1 < c1 and d[p+1] != '\n' starts a match (seen = true); its end is 1 + the first
 * '\n' at or after p in the WHOLE object, or the object size (the seek+readline fix-up, fasta.py:45-56).
 */
#include <stdint.h>
#include <string.h>

static uint64_t next_nl_end(const uint8_t* d, uint64_t size, uint64_t p) {
  const uint8_t* q = (const uint8_t*)memchr(d + p, '\n', size - p);
  return q ? (uint64_t)(q - d) + 1 : size;
}

/* returns the number of pairs; writes min(cap, pairs) interleaved (start, end) uint64 values */
int64_t dpref_fasta(const uint8_t* d, uint64_t size, const uint64_t* chunks, uint64_t nchunks, uint64_t* out,
                    uint64_t cap) {
  uint64_t n = 0;
  for (uint64_t c = 0; c < nchunks; ++c) {
    const uint64_t c0 = chunks[2 * c], c1 = chunks[2 * c + 1];
    uint64_t p = c0;
    while (p < c1) {
      /* next '>' in the chunk */
      const uint8_t* g = (const uint8_t*)memchr(d + p, '>', c1 - p);
      if (!g) break;
      const uint64_t s = (uint64_t)(g - d);
      if (s + 1 < c1 && d[s + 1] != '\n') {
        const uint64_t e = next_nl_end(d, size, s);
        if (n < cap) {
          out[2 * n] = s;
          out[2 * n + 1] = e;
        }
        ++n;
        p = e;                        /* the match consumed the rest of the line (seen until '\n') */
      } else {
        p = s + 1;                    /* '>' at the chunk end or right before '\n': no match */
      }
    }
  }
  return (int64_t)n;
}

/* offsets of every every_k-th `delim` in [begin, end) plus emit_add; returns the number of entries */
int64_t dpref_delim(const uint8_t* d, uint64_t begin, uint64_t end, uint32_t delim, uint32_t every_k,
                    uint32_t emit_add, uint64_t* out, uint64_t cap, uint64_t* ndelims) {
  uint64_t g = 0, n = 0, p = begin;
  while (p < end) {
    const uint8_t* q = (const uint8_t*)memchr(d + p, (int)delim, end - p);
    if (!q) break;
    const uint64_t s = (uint64_t)(q - d);
    if (g % every_k == every_k - 1) {
      if (n < cap) out[n] = s + emit_add;
      ++n;
    }
    ++g;
    p = s + 1;
  }
  if (ndelims) *ndelims = g;
  return (int64_t)n;
}
