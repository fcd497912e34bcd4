// dpscan.hip — MI355X (gfx950, CDNA4) record-boundary scan kernels + the C ABI of libdpscan.so.
//
// What runs here:
//   * scan_kernel<FASTA>: the FASTA header index of dataplug/formats/genomics/fasta.py:24-63 for a whole
//     chunk plan in ONE pass over HBM; emits (start, end) offset pairs bit-exact to the reference.
//   * scan_kernel<DELIM>: sorted offsets of a delimiter byte (CSV/VCF newline index, FASTQ read ends).
//   * fasta_resolve_kernel / find_kernel: the "header cut by the chunk end" fix-up (fasta.py:45-56).
//
// Single pass, memory-bound (no MFMA):
//   * persistent grid, one 1024-thread workgroup per CU = 15 data waves + 1 coordinator wave; the
//     workgroup owns the 120 KiB units u = blockIdx.x + k*G (each data wave 8 rows of 1 KiB = 64 lanes
//     x 16 B bounds-checked buffer loads, double-buffered in VGPRs, hand-waited).
//   * per 16-byte lane: SWAR exact byte matches packed into one interleaved 32-bit mask ('\n' at even,
//     '>' at odd bits), a carry trick that marks the first valid '>' of every line segment, and the
//     lane-level line state from one 64-bit carry trick on the wave's ballots (SGPRs).
//   * phase A summarises a wave's 8 KiB as a FUNCTION of the incoming line state and parks its masks in
//     LDS; the coordinator chains unit summaries across workgroups with a decoupled look-back over
//     8-byte {status, value} descriptors (agent-scope relaxed atomics = sc1; cdna_hip_programming.md G16
//     R2) and hands prefixes back through LDS flags; phase B turns masks into offsets.  Input bytes are
//     read from HBM exactly once; data waves never wait on each other (no workgroup barrier per unit).
//   * every wait is bounded (DP_ERR_TIMEOUT); units are statically strided over a grid of one
//     workgroup per CU, so a unit only ever waits on lower units owned by running workgroups.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <type_traits>
#include <vector>

#include "../../include/dpscan.h"

namespace {

constexpr int kWave = 64;
constexpr int kDataWaves = 15;                     // + 1 coordinator wave
constexpr int kCoord = kDataWaves;
constexpr int kWaves = kDataWaves + 1;
constexpr int kThreads = kWave * kWaves;           // 1024
constexpr int kRowBytes = kWave * 16;              // one dwordx4 per lane
constexpr int kRows = 8;                           // rows per wave per unit
constexpr int kWaveBytes = kRowBytes * kRows;      // 8 KiB
constexpr int kUnitBytes = kWaveBytes * kDataWaves;  // 120 KiB look-back unit
#ifndef DP_RING
#define DP_RING 4
#endif
#ifndef DP_PRIO
#define DP_PRIO 1
#endif
#ifndef DP_STEAL            // phase-B tasks shared by all data waves (else each wave runs its own, lagged)
#define DP_STEAL 0
#endif
#ifndef DP_WAVEPUB          // the last data wave of a unit composes and publishes its AGG (else the coordinator)
#define DP_WAVEPUB 0
#endif
#ifndef DP_LBPREFETCH       // the coordinator prefetches the next unit's look-back window
#define DP_LBPREFETCH 1
#endif
constexpr int kRing = DP_RING;                     // LDS ring depth (units in flight per workgroup)
constexpr int kLag = 2;                            // resolve(j) once unit j + kLag is composed (its AGG out)
[[maybe_unused]] constexpr int kBLag = kRing - 1;  // !DP_STEAL: data waves run phase B(j) after phase A(j + kBLag)
static_assert(kLag < kRing, "slot j + kLag must still hold that unit when the coordinator waits on it");
constexpr uint32_t kGT = 0x3E3E3E3Eu;              // '>'
constexpr uint32_t kNL = 0x0A0A0A0Au;              // '\n'
constexpr uint32_t kOdd = 0xAAAAAAAAu, kEven = 0x55555555u;

constexpr uint32_t kErrTimeout = 1u;
constexpr uint32_t kErrOverflow = 2u;

constexpr uint64_t kStatAgg = 1ull << 62;
constexpr uint64_t kStatPrefix = 2ull << 62;
constexpr uint64_t kStatMask = 3ull << 62;
constexpr uint32_t kSpinLimit = 1u << 22;          // polls (with s_sleep) before giving up

enum Mode { kFasta = 0, kDelim = 1 };

// In-kernel section timers (diagnostics build only: -DDP_PROF).  Per workgroup and wave, kProfSlots
// accumulated s_memtime deltas; read back with dp_debug_profile().
#ifdef DP_PROF
constexpr int kProfSlots = 8;
constexpr int kProfWaves = 16;
constexpr int kProfMaxGrid = 1024;
__device__ unsigned long long g_prof[kProfMaxGrid * kProfWaves * kProfSlots];
#define PROF_DECL uint64_t prof_acc[kProfSlots] = {0, 0, 0, 0, 0, 0, 0, 0}; uint64_t prof_t = __builtin_amdgcn_s_memtime()
#define PROF_MARK(slot) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); prof_acc[slot] += t_ - prof_t; prof_t = t_; } while (0)
#define PROF_FLUSH(wave) do { if (__lane_id() == 0 && blockIdx.x < kProfMaxGrid) { for (int i_ = 0; i_ < kProfSlots; ++i_) \
    g_prof[((uint64_t)blockIdx.x * kProfWaves + (wave)) * kProfSlots + i_] = prof_acc[i_]; } } while (0)
#define PROF_ARG , uint64_t (&prof_acc)[kProfSlots], uint64_t& prof_t
#define PROF_PASS , prof_acc, prof_t
#else
#define PROF_DECL do {} while (0)
#define PROF_MARK(slot) do {} while (0)
#define PROF_FLUSH(wave) do {} while (0)
#define PROF_ARG
#define PROF_PASS
#endif

struct ScanArgs {
  const uint8_t* base;         // 16-byte aligned base; coordinates below are relative to it
  uint64_t shift;              // buffer start - base (0..15)
  uint64_t obj_base;           // object offset of buffer byte 0
  uint64_t nchunks;
  uint64_t nunits;
  unsigned long long* desc;    // [nunits] look-back descriptors (zeroed per launch)
  void* out;
  uint64_t cap;                // entries (FASTA: pairs)
  int out_u64;
  uint32_t delim;              // DELIM: byte replicated x4
  uint32_t every_k;
  uint32_t emit_add;
  uint32_t* err;
  unsigned long long* total;   // inclusive count at the last unit
  long long* pending;          // FASTA: [nchunks] pair index whose end is unresolved at chunk end, or -1
  unsigned long long* chunk_end;  // [nchunks] inclusive count at the end of each (non-empty) chunk
};

// ------------------------------------------------------------------------------------------ helpers
__device__ __forceinline__ uint32_t eq4(uint32_t w, uint32_t pat) {
  // exact: bit 8j+7 set iff byte j of w equals the pattern byte
  const uint32_t x = w ^ pat;
  const uint32_t t = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return ~(t | x) & 0x80808080u;
}
// v_mul_u32_u24 with a literal multiplier.  The compiler otherwise hoists the constant into an SGPR and
// emits the quarter-rate v_mul_lo_u32.
template <uint32_t K>
__device__ __forceinline__ uint32_t mul24k(uint32_t a) {
  uint32_t r;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "i"(K), "v"(a));
  return r;
}
__device__ __forceinline__ uint32_t pack4(uint32_t e) {
  // bits 7,15,23,31 -> bits 0..3 (mul_u32_u24 gather)
  const uint32_t f = e >> 7;
  return ((mul24k<0x4081u>(f & 0x10101u) >> 14) & 7u) | (f >> 21);
}
__device__ __forceinline__ uint32_t mask16(const uint4& v, uint32_t pat) {
  return pack4(eq4(v.x, pat)) | (pack4(eq4(v.y, pat)) << 4) | (pack4(eq4(v.z, pat)) << 8) |
         (pack4(eq4(v.w, pat)) << 12);
}
// 4 bytes -> 8 interleaved flags: bit 2j = (byte j == '\n'), bit 2j+1 = (byte j == '>').  The pairs of
// bytes 0..2 are gathered by one mul_u32_u24 (partial products land on disjoint bits: no carries).
__device__ __forceinline__ uint32_t pair8(uint32_t w) {
  const uint32_t c = (eq4(w, kGT) | (eq4(w, kNL) >> 1)) >> 6;   // byte j: bit 8j = nl, 8j+1 = gt
  const uint32_t t = (mul24k<0x41041u>(c & 0x30303u) >> 18) & 0x3Fu;
  return t | ((c >> 18) & 0xC0u);
}
__device__ __forceinline__ uint32_t pairs32(const uint4& v) {
  return pair8(v.x) | (pair8(v.y) << 8) | (pair8(v.z) << 16) | (pair8(v.w) << 24);
}
__device__ __forceinline__ bool maybe_has(const uint4& v, uint32_t pat) {
  // no false negatives (classic haszero); false positives only make the exact path run
  auto hz = [](uint32_t x) { return (x - 0x01010101u) & ~x; };
  return ((hz(v.x ^ pat) | hz(v.y ^ pat) | hz(v.z ^ pat) | hz(v.w ^ pat)) & 0x80808080u) != 0;
}
// bytes [a, b) of a 16-byte lane (a, b clamped to 0..16) as 16 single / 32 paired bits
__device__ __forceinline__ uint32_t range16(int64_t a, int64_t b) {
  a = a < 0 ? 0 : (a > 16 ? 16 : a);
  b = b < 0 ? 0 : (b > 16 ? 16 : b);
  return b <= a ? 0u : ((0xFFFFu >> (16 - (b - a))) << a);
}
__device__ __forceinline__ uint32_t range32(int64_t a, int64_t b) {
  a = a < 0 ? 0 : (a > 16 ? 16 : a);
  b = b < 0 ? 0 : (b > 16 ? 16 : b);
  return b <= a ? 0u : (uint32_t)((0xFFFFFFFFull >> (32 - 2 * (b - a))) << (2 * a));
}
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// exclusive wave prefix + total of small per-lane counts (< 2^BITS), bit-sliced ballots
template <int BITS>
__device__ __forceinline__ uint32_t wave_excl(uint32_t c, uint32_t& total) {
  const uint64_t any1 = __ballot(c != 0u);
  if (__ballot(c > 1u) == 0ull) {                    // common: at most one per lane
    total = (uint32_t)__popcll(any1);
    return mbcnt(any1);
  }
  uint32_t ex = 0, tot = 0;
#pragma unroll
  for (int b = 0; b < BITS; ++b) {
    const uint64_t m = __ballot((c >> b) & 1u);
    ex += mbcnt(m) << b;
    tot += (uint32_t)__popcll(m) << b;
  }
  total = tot;
  return ex;
}
template <int BITS>
__device__ __forceinline__ uint32_t wave_total(uint32_t c) {
  const uint64_t any2 = __ballot(c > 1u);
  const uint64_t any1 = __ballot(c != 0u);
  if (!any2) return (uint32_t)__popcll(any1);        // common: at most one per lane
  uint32_t tot = 0;
#pragma unroll
  for (int b = 0; b < BITS; ++b) tot += (uint32_t)__popcll(__ballot((c >> b) & 1u)) << b;
  return tot;
}
__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)x, l);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t rfl(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t ld_desc(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_desc(unsigned long long* p, uint64_t v) {
  __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// LDS hand-offs inside the workgroup.  LDS executes one wave's operations in order, so a relaxed flag
// written after the payload (with a compiler barrier in between) is seen after it; no global fence
// (which would make the data waves drain their in-flight prefetch).
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_add(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void cbar() { asm volatile("" ::: "memory"); }

// Issue priority (s_setprio takes an immediate).  The 4 data waves sharing a SIMD (w, w+4, w+8, w+12)
// otherwise get issue slots by age: the youngest is starved, and as every unit waits for its slowest
// wave the older ones idle.  Rotating the priority per unit gives each wave every rank once in 4 units.
__device__ __forceinline__ void set_prio(uint32_t p) {
#if DP_PRIO
  switch (p & 3u) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
  }
#else
  (void)p;
#endif
}

// Summary of a byte range as a function of the incoming line state S (does the current line already
// hold an emitted header?): count and outgoing state for S = false (F) and S = true (T).
struct Func {
  uint64_t cF, cT;
  uint32_t sF, sT;
};
__device__ __forceinline__ Func f_then(const Func& a, const Func& b) {   // a, then b
  const uint64_t bF = b.cF, bT = b.cT;
  const uint32_t bsF = b.sF, bsT = b.sT;
  const uint32_t mF = 0u - (a.sF & 1u), mT = 0u - (a.sT & 1u);
  const uint64_t mF64 = 0ull - (uint64_t)(a.sF & 1u), mT64 = 0ull - (uint64_t)(a.sT & 1u);
  Func r;
  r.cF = a.cF + ((bT & mF64) | (bF & ~mF64));
  r.sF = (bsT & mF) | (bsF & ~mF);
  r.cT = a.cT + ((bT & mT64) | (bF & ~mT64));
  r.sT = (bsT & mT) | (bsF & ~mT);
  return r;
}
__device__ __forceinline__ uint64_t pack_agg(const Func& f) {
  return kStatAgg | ((uint64_t)f.sT << 49) | ((uint64_t)f.sF << 48) | ((f.cT & 0xFFFFFFull) << 24) |
         (f.cF & 0xFFFFFFull);
}
__device__ __forceinline__ uint64_t pack_prefix(uint64_t count, uint32_t s) {
  return kStatPrefix | ((uint64_t)s << 48) | (count & 0xFFFFFFFFFFFFull);
}

template <typename T>
__device__ __forceinline__ void put(void* out, uint64_t i, uint64_t v) {
  reinterpret_cast<T*>(out)[i] = (T)v;
}

// ------------------------------------------------------------------------------------------ look-back
// Unit summaries in the decoupled look-back carry an "inclusive prefix" flag: a PREFIX descriptor is a
// constant function (it already counts everything before it), so composing anything in front of it
// yields it unchanged.  lb_then() is associative, which lets a wave reduce a whole window in a tree.
struct LB {
  uint64_t cF, cT;
  uint32_t fl;     // bit0 sF, bit1 sT, bit2 inclusive prefix
};
__device__ __forceinline__ LB lb_ident() { return LB{0, 0, 2u}; }
// mask selects: `c ? x : y` on struct members otherwise becomes an indexed stack copy (scratch)
__device__ __forceinline__ uint64_t sel64(uint32_t c, uint64_t x, uint64_t y) {
  const uint64_t m = 0ull - (uint64_t)(c & 1u);
  return (x & m) | (y & ~m);
}
__device__ __forceinline__ uint32_t sel32(uint32_t c, uint32_t x, uint32_t y) {
  const uint32_t m = 0u - (c & 1u);
  return (x & m) | (y & ~m);
}
__device__ __forceinline__ LB lb_then(const LB& a, const LB& b) {   // a (farther), then b (nearer)
  const uint32_t asF = a.fl & 1u, asT = (a.fl >> 1) & 1u;
  const uint32_t bsF = b.fl & 1u, bsT = (b.fl >> 1) & 1u;
  const uint32_t bp = (b.fl >> 2) & 1u;              // b is an inclusive prefix: absorbs a
  const uint64_t bF = b.cF, bT = b.cT;
  LB r;
  r.cF = sel64(bp, bF, a.cF + sel64(asF, bT, bF));
  r.cT = sel64(bp, bT, a.cT + sel64(asT, bT, bF));
  r.fl = sel32(bp, b.fl, sel32(asF, bsT, bsF) | (sel32(asT, bsT, bsF) << 1) | (a.fl & 4u));
  return r;
}
__device__ __forceinline__ LB lb_from_desc(uint64_t d) {
  const uint64_t st = d & kStatMask;
  if (st == kStatAgg) return LB{d & 0xFFFFFFull, (d >> 24) & 0xFFFFFFull, (uint32_t)(d >> 48) & 3u};
  if (st == kStatPrefix) {
    const uint64_t c = d & 0xFFFFFFFFFFFFull;
    const uint32_t s = (uint32_t)(d >> 48) & 1u;
    return LB{c, c, s | (s << 1) | 4u};
  }
  return lb_ident();
}

// DPP lane moves (VALU, no LDS round trip).  Lanes whose source is outside the pattern get `old`.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp32(uint32_t x, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, CTRL, ROWS, 0xF, false);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp64(uint64_t x, uint64_t old) {
  return ((uint64_t)dpp32<CTRL, ROWS>((uint32_t)(x >> 32), (uint32_t)(old >> 32)) << 32) |
         dpp32<CTRL, ROWS>((uint32_t)x, (uint32_t)old);
}
constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118;
constexpr int kRowBcast15 = 0x142, kRowBcast31 = 0x143;   // gfx9 DPP: lane 15 / 31 to the next row(s)

template <int CTRL, int ROWS>
__device__ __forceinline__ LB lb_dpp(const LB& f) {       // identity where there is no source lane
  LB o;
  o.cF = dpp64<CTRL, ROWS>(f.cF, 0ull);
  o.cT = dpp64<CTRL, ROWS>(f.cT, 0ull);
  o.fl = dpp32<CTRL, ROWS>(f.fl, 2u);
  return o;
}
template <int CTRL, int ROWS>
__device__ __forceinline__ Func fn_dpp(const Func& f) {
  Func o;
  o.cF = dpp64<CTRL, ROWS>(f.cF, 0ull);
  o.cT = dpp64<CTRL, ROWS>(f.cT, 0ull);
  o.sF = dpp32<CTRL, ROWS>(f.sF, 0u);
  o.sT = dpp32<CTRL, ROWS>(f.sT, 1u);
  return o;
}

constexpr uint64_t kIdentDesc = kStatMask;   // status 3: "no unit here" (identity, always valid)

// One wave: prefix count P and line state S entering unit u.  The window is every unit between this
// workgroup's previous unit (u - G, whose inclusive prefix the coordinator holds in registers) and u,
// all published by running workgroups: one parallel load (4 descriptors per lane for G <= 256) and a
// 6-step ordered tree reduction resolve it — no serial chain of prefixes.  Spins are bounded.
// First window of descriptors for unit u (lane 63 = nearest): D[k] = desc[u-1-k] for k < W, D[W] = the
// workgroup's own previous unit's inclusive prefix (base), identity past it.
__device__ __forceinline__ void lb_load(const ScanArgs& A, uint64_t u, uint64_t G, uint64_t k0, uint64_t basedesc,
                                        int lane, uint64_t (&d)[4]) {
  const uint64_t W = u < G - 1 ? u : G - 1;
  const int rl = kWave - 1 - lane;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint64_t k = k0 + 4 * (uint64_t)rl + j;
    d[j] = k < W ? ld_desc(&A.desc[u - 1 - k]) : (k == W ? basedesc : kIdentDesc);
  }
}

// One wave: prefix count P and line state S entering unit u.  The window is every unit between this
// workgroup's previous unit (u - G, whose inclusive prefix the coordinator holds in registers) and u,
// all published by running workgroups: one parallel load (4 descriptors per lane for G <= 256; the
// caller may pass it in already loaded, `pre`) and a DPP scan resolve it — no serial chain of prefixes.
// Spins are bounded.
__device__ __forceinline__ void lookback(const ScanArgs& A, uint64_t u, uint64_t G, uint64_t baseP, uint32_t baseS,
                                      int lane, uint64_t& P, uint32_t& S_in, uint64_t (&pre)[4], bool have_pre
                                      PROF_ARG) {
  const uint64_t basedesc = pack_prefix(baseP, baseS);
  LB acc = lb_ident();
  for (uint64_t k0 = 0;; k0 += 4 * kWave) {
    uint64_t d[4];
    uint64_t PB;
    uint32_t spins = 0;
    if (k0 == 0 && have_pre) {
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = pre[j];
    } else {
      lb_load(A, u, G, k0, basedesc, lane, d);
    }
    for (;;) {
      uint32_t seen = 0, bad = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {                   // nearest first
        const uint64_t st = d[j] & kStatMask;
        if (!seen && st == 0ull) bad = 1;
        if (st == kStatPrefix) seen = 1;
      }
      PB = __ballot(seen);
      const uint64_t BB = __ballot(bad);
      // lanes from the nearest one (63) down to the nearest lane holding a prefix must all be published
      const uint64_t need = PB ? ~((1ull << (63 - __builtin_clzll(PB))) - 1ull) : ~0ull;
      if ((BB & need) == 0ull) break;
      if (++spins > kSpinLimit) {
        if (lane == 0) atomicOr(A.err, kErrTimeout);
        d[0] = pack_prefix(0, 0);
        d[1] = d[2] = d[3] = kIdentDesc;
        PB = 1ull;
        break;
      }
      __builtin_amdgcn_s_sleep(8);                    // back off: reloads compete with the stream
      lb_load(A, u, G, k0, basedesc, lane, d);
#ifdef DP_PROF
      prof_acc[4] += 1;                               // spin count (not time)
#endif
    }
    PROF_MARK(6);                                     // first valid window (load latency + spins)
    LB f = lb_from_desc(d[3]);
    f = lb_then(f, lb_from_desc(d[2]));
    f = lb_then(f, lb_from_desc(d[1]));
    f = lb_then(f, lb_from_desc(d[0]));
    // inclusive scan, lane 0 (farthest) -> lane 63 (nearest): farther composed in front of nearer
    f = lb_then(lb_dpp<kRowShr1, 0xF>(f), f);
    f = lb_then(lb_dpp<kRowShr2, 0xF>(f), f);
    f = lb_then(lb_dpp<kRowShr4, 0xF>(f), f);
    f = lb_then(lb_dpp<kRowShr8, 0xF>(f), f);
    f = lb_then(lb_dpp<kRowBcast15, 0xA>(f), f);
    f = lb_then(lb_dpp<kRowBcast31, 0xC>(f), f);
    LB F;
    F.cF = readlane64(f.cF, kWave - 1);
    F.cT = readlane64(f.cT, kWave - 1);
    F.fl = (uint32_t)__builtin_amdgcn_readlane((int)f.fl, kWave - 1);
    acc = lb_then(F, acc);
    if (PB) break;
  }
  P = acc.cF;
  S_in = acc.fl & 1u;
}

// ------------------------------------------------------------------------------------------ geometry
// Unit -> chunk lookup over the chunk table (read-only, read through the constant address space so it
// compiles to scalar loads and never enters the vector-memory counter the data waves' hand-waited loads
// rely on).  A cursor follows
// the increasing units of one wave, falling back to a binary search when it would skip chunks.
typedef __attribute__((address_space(4))) const uint64_t cu64;   // constant address space: s_load
struct Tab {
  cu64* lo;
  cu64* hi;
  cu64* u0;                          // [nchunks + 1]
};
struct Cursor {
  uint64_t c, u0, u1, lo, hi;        // chunk c = [lo, hi) covers units [u0, u1)
  uint32_t valid;
};
struct Geo {                          // one unit (wave-uniform)
  uint64_t lo, hi, ubase, c;
  uint32_t first, last, valid;
};
__device__ __forceinline__ Geo geo_of(const Tab& T, uint64_t nchunks, uint64_t nunits, uint64_t u, Cursor& cur) {
  Geo g;
  if (u >= nunits) {
    g.lo = g.hi = g.ubase = g.c = 0;
    g.first = g.last = g.valid = 0;
    return g;
  }
  if (!cur.valid || u < cur.u0 || u >= cur.u1) {
    uint64_t c = 0, cn = nchunks;
    if (cur.valid && u >= cur.u1 && cur.c + 1 < nchunks && T.u0[cur.c + 2] > u) {
      c = cur.c + 1;                                   // common case: the next chunk
    } else {
      while (cn - c > 1) {
        const uint64_t m = (c + cn) >> 1;
        if (T.u0[m] <= u) c = m; else cn = m;
      }
    }
    cur.c = c;
    cur.u0 = T.u0[c];
    cur.u1 = T.u0[c + 1];
    cur.lo = T.lo[c];
    cur.hi = T.hi[c];
    cur.valid = 1;
  }
  g.c = cur.c;
  g.lo = cur.lo;
  g.hi = cur.hi;
  g.first = (u == cur.u0);
  g.last = (u + 1 == cur.u1);
  g.valid = 1;
  g.ubase = (g.lo & ~15ull) + (u - cur.u0) * (uint64_t)kUnitBytes;
  return g;
}

// ------------------------------------------------------------------------------------------ input loads
typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

struct Buf {
  v4u x[kRows];              // raw load destinations (owned by the in-flight asm loads until wait_buf)
  uint32_t la;               // first dword after this wave's range (next-byte lookahead of row 7)
};

// Unconditional bounds-checked loads of one wave's 8 KiB (+ lookahead): bytes at or past the 16-byte
// block holding the chunk end read as 0 (num_records), so every wave always has exactly kLoadsPerBuf
// loads in flight per buffer.  Issued as inline asm: the compiler inserts no wait for them, and the
// data waves wait with ONE explicit `s_waitcnt vmcnt(kLoadsPerBuf)` at the top of phase A (the only
// younger vector-memory ops are the other buffer's loads plus stores, which only make it conservative).
// tools/isa_guard.py checks the compiled code never touches a destination before that wait.
constexpr int kLoadsPerBuf = kRows + 1;

__device__ __forceinline__ void load_buf(Buf& b, const ScanArgs& A, const Geo& g, int wave, int lane) {
  const uint64_t wbase = g.valid ? g.ubase + (uint64_t)wave * kWaveBytes : 0ull;
  const uint64_t hi16 = (g.hi + 15) & ~15ull;
  uint32_t nrec = 0;
  if (g.valid && hi16 > wbase) nrec = (uint32_t)((hi16 - wbase) < (uint64_t)(kWaveBytes + 16) ? (hi16 - wbase) : (kWaveBytes + 16));
  const uint64_t addr = (uint64_t)(uintptr_t)(A.base + wbase);
  v4i r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)addr);
  r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(addr >> 32) & 0xFFFF);   // stride 0
  r[2] = __builtin_amdgcn_readfirstlane((int)nrec);
  r[3] = 0x00020000;
  const uint32_t off0 = (uint32_t)lane * 16u, off1 = off0 + 4096u, offla = (uint32_t)kWaveBytes;
  static_assert(kRows == 8 && kRowBytes == 1024, "load_buf offsets assume 8 rows of 1 KiB");
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:0" : "=v"(b.x[0]) : "v"(off0), "s"(r) : "memory");
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:1024" : "=v"(b.x[1]) : "v"(off0), "s"(r) : "memory");
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:2048" : "=v"(b.x[2]) : "v"(off0), "s"(r) : "memory");
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:3072" : "=v"(b.x[3]) : "v"(off0), "s"(r) : "memory");
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:0" : "=v"(b.x[4]) : "v"(off1), "s"(r) : "memory");
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:1024" : "=v"(b.x[5]) : "v"(off1), "s"(r) : "memory");
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:2048" : "=v"(b.x[6]) : "v"(off1), "s"(r) : "memory");
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:3072" : "=v"(b.x[7]) : "v"(off1), "s"(r) : "memory");
  asm volatile("buffer_load_dword %0, %1, %2, 0 offen" : "=v"(b.la) : "v"(offla), "s"(r) : "memory");
}

// Wait for this buffer's loads, then "redefine" every destination register: the empty asm makes each
// value live until here (an unused destination must not be reallocated while its load is in flight)
// and nothing that reads the data can be scheduled above the wait.
__device__ __forceinline__ void touch_buf(Buf& b) {
  asm volatile("" : "+v"(b.x[0]), "+v"(b.x[1]), "+v"(b.x[2]), "+v"(b.x[3]), "+v"(b.x[4]), "+v"(b.x[5]),
               "+v"(b.x[6]), "+v"(b.x[7]), "+v"(b.la) :: "memory");
}
__device__ __forceinline__ void wait_buf(Buf& b) {
  asm volatile("s_waitcnt vmcnt(%0)" :: "i"(kLoadsPerBuf) : "memory");
  touch_buf(b);
  __builtin_amdgcn_sched_barrier(0);
}
// After the last step both buffers still have (unused) loads in flight: wait for them and keep their
// destinations live until then, or the compiler reuses those VGPRs and the landing loads clobber them.
__device__ __forceinline__ void drain_bufs(Buf& a, Buf& b) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  touch_buf(a);
  touch_buf(b);
  __builtin_amdgcn_sched_barrier(0);
}

// ------------------------------------------------------------------------------------------ LDS state
// Phase-B state of a unit (wave-uniform; the per lane-row masks wait in LDS too: FASTA interleaved
// emits (odd bits) | ends (even bits), DELIM delimiter bits).
struct Pend {
  uint64_t wbase;
  uint32_t rows;             // bit r: row r has a nonzero mask in some lane
  uint32_t fV;               // FASTA: first segment of the wave range held a valid '>'
  int fn_off;                // FASTA: first '\n' of the wave range (byte offset in the range) or -1
  uint32_t pad;
};

struct Shared {
  uint64_t cF[kRing][kDataWaves], cT[kRing][kDataWaves];   // per-wave summaries
  uint32_t sF[kRing][kDataWaves], sT[kRing][kDataWaves];
  uint64_t exF[kRing][kDataWaves], exT[kRing][kDataWaves];  // per-wave exclusive prefix functions (coordinator)
  uint32_t esF[kRing][kDataWaves], esT[kRing][kDataWaves];
  uint64_t uF[kRing], uT[kRing];                            // the unit's function
  uint32_t usF[kRing], usT[kRing];
  uint64_t P[kRing][kDataWaves];                           // per-wave prefixes from the coordinator
  uint32_t S[kRing][kDataWaves];
  uint32_t done[kRing];                                    // data waves finished phase A of the slot's unit
  uint32_t composed[kRing];                                // = unit index + 1 once its AGG is composed/published
  uint32_t ready[kRing];                                   // = unit index + 1 once P/S of the slot are set
  uint32_t bclaim;                                         // phase-B tasks handed out (task = unit*15 + wave)
  uint32_t bdone[kRing];                                   // phase-B tasks finished per slot (monotonic)
  Pend pend[kRing][kDataWaves];
  uint32_t m[kRing][kDataWaves][kRows][kWave];             // 120 KiB
};

// ------------------------------------------------------------------------------------------ FASTA row
// One row (64 lanes x 16 bytes) under the wave-uniform incoming line state S.  Interleaved masks:
// bit 2i = byte i is '\n', bit 2i+1 = byte i is a valid '>' (followed by a non-'\n' byte inside the chunk).
struct FRow {
  uint32_t m;                // emits (odd bits) | ends (even bits)
  uint32_t nemit;            // emits in this lane
  uint32_t s_before_nl;      // line state just before this lane's first '\n'
  uint32_t first_nl;         // bit index (even) of this lane's first '\n', or 32
  uint64_t H;                // ballot: lanes holding a '\n'
  uint32_t S_out;            // wave-uniform state after the row
};
__device__ __forceinline__ FRow fasta_row(uint32_t M, uint32_t nxt63, int last_bit, uint32_t S, int lane) {
  FRow f;
  const uint32_t NL = M & kEven, GT = M & kOdd;
  // next lane's byte 0 is '\n'? (wave_shl:1 DPP; lane 63 takes the lookahead byte)
  const uint32_t nb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(NL & 1u), 0x130, 0xF, 0xF, false);
  const uint32_t nxt = (lane == kWave - 1) ? nxt63 : nb;
  uint32_t V = GT & ~((NL >> 1) | (nxt << 31));      // '>' followed by a non-'\n' byte
  if (last_bit >= 0) V &= ~(1u << last_bit);          // p + 1 < c1
  const uint32_t X = V | NL;
  // first X bit at/after every line start (lane start, byte after each '\n'): carries run through ~X
  const uint64_t R64 = (uint64_t)(~X) + ((((uint64_t)NL) << 2) | 1ull);
  const uint32_t R = (uint32_t)R64;
  const uint32_t s_last = (uint32_t)(R64 >> 32) ^ 1u;    // a valid '>' after the lane's last '\n'
  const uint64_t H = __ballot(NL != 0u);
  const uint64_t SB = __ballot(s_last);
  // line state at each lane's start: exit(p) = H(p) ? SB(p) : exit(p-1) | SB(p), start(0) = S — a
  // carry chain over the 64 lanes: generate = SB, propagate = ~H (wave-uniform, scalar unit)
  const uint64_t a = SB | ~H;
  const uint64_t s1 = a + SB;
  const uint64_t c1 = s1 < a;
  const uint64_t s2 = s1 + (uint64_t)S;
  const uint64_t c2 = s2 < s1;
  const uint64_t Sstart = s2 ^ a ^ SB;
  f.S_out = (uint32_t)(c1 | c2);
  const uint32_t S_lane = (uint32_t)((Sstart >> lane) & 1ull);
  const uint32_t low = NL & (0u - NL);
  const uint32_t fs = low ? low - 1u : 0xFFFFFFFFu;   // bits before the lane's first '\n'
  const uint32_t emits = V & R & (S_lane ? ~fs : 0xFFFFFFFFu);
  const uint32_t ends = NL & (~R | (S_lane ? low : 0u));
  f.m = emits | ends;
  f.nemit = (uint32_t)__popc(emits);
  f.s_before_nl = S_lane | ((V & fs) != 0u);
  f.first_nl = low ? (uint32_t)__builtin_ctz(low) : 32u;
  f.H = H;
  return f;
}

// ------------------------------------------------------------------------------------------ phase A / B
// Phase A of one unit on one data wave: masks (to LDS) + the wave's summary as a function of the
// incoming line state (hypothesis: the wave's range starts with S = false).
template <int MODE>
__device__ __forceinline__ Func phase_a(const ScanArgs& A, const Geo& g, Buf& b, Pend& p, uint32_t (&ms)[kRows][kWave],
                                        int lane, int wave PROF_ARG) {
  uint64_t cnt = 0;
  uint32_t S = 0, nlseen = 0, fV = 0;
  int fn_off = -1;
  const uint64_t lo = g.lo, hi = g.hi;
  const uint64_t wbase = g.ubase + (uint64_t)wave * kWaveBytes;
  uint32_t rows = 0;
  wait_buf(b);                                       // this buffer landed; the other one stays in flight
  PROF_MARK(0);
  uint4 v[kRows];
#pragma unroll
  for (int r = 0; r < kRows; ++r) v[r] = make_uint4(b.x[r][0], b.x[r][1], b.x[r][2], b.x[r][3]);
  const uint32_t la = b.la;
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    const uint64_t row0 = wbase + (uint64_t)r * kRowBytes;
    if (!g.valid || row0 >= hi) continue;
    // edge row: touches the chunk start, or holds the chunk's last byte (never a header: p+1 < c1)
    const bool edge = row0 < lo || row0 + kRowBytes >= hi;
    const int64_t rel_lo = (int64_t)lo - (int64_t)row0 - 16 * lane;   // chunk bounds relative to the lane
    const int64_t rel_hi = (int64_t)hi - (int64_t)row0 - 16 * lane;
    uint32_t mr;
    if constexpr (MODE == kFasta) {
      if (!S && nlseen && __ballot(maybe_has(v[r], kGT)) == 0ull) continue;
      uint32_t nxt = 0;
      if (row0 + kRowBytes < hi) {
        const uint32_t w = (r + 1 < kRows) ? v[(r + 1) & (kRows - 1)].x : la;
        nxt = ((uint32_t)__builtin_amdgcn_readlane((int)w, 0) & 0xFFu) == 10u;
      }
      uint32_t M = pairs32(v[r]);
      int last_bit = -1;
      if (edge) {
        M &= range32(rel_lo, rel_hi);
        last_bit = (rel_hi >= 1 && rel_hi <= 16) ? (int)(2 * (rel_hi - 1) + 1) : -1;
      }
      const FRow f = fasta_row(M, nxt, last_bit, S, lane);
      if (!nlseen && f.H) {
        const int j0 = (int)__builtin_ctzll(f.H);
        fV = __builtin_amdgcn_readlane((int)f.s_before_nl, j0);
        fn_off = r * kRowBytes + j0 * 16 + (int)(__builtin_amdgcn_readlane((int)f.first_nl, j0) >> 1);
        nlseen = 1;
      }
      mr = f.m;
      cnt += wave_total<3>(f.nemit);
      S = f.S_out;
    } else {
      mr = mask16(v[r], A.delim);
      if (edge) mr &= range16(rel_lo, rel_hi);
      cnt += wave_total<5>((uint32_t)__popc(mr));
    }
    if (__ballot(mr != 0u)) {
      rows |= 1u << r;
      ms[r][lane] = mr;
    }
  }
  Func ws;
  if constexpr (MODE == kFasta) {
    if (!nlseen) fV = S;
    ws = Func{cnt, cnt - fV, S, nlseen ? S : 1u};
    if (g.first && wave == 0) { ws.cT = ws.cF; ws.sT = ws.sF; }
  } else {
    ws = Func{cnt, cnt, 0u, 0u};
  }
  p.wbase = wbase;
  p.rows = rows;
  p.fV = fV;
  p.fn_off = fn_off;
  p.pad = 0;
  PROF_MARK(1);
  return ws;
}

// Phase B: offsets from the masks, given the wave's true prefix count and incoming line state.
// Stores go to min(index, cap - 1) (the host guarantees cap >= 1): an overflowing launch reports
// DP_ERR_CAPACITY and its output is discarded, so the clamp replaces a per-store branch.  The uint32
// overflow check (offset >= 2^32) only runs in rows whose offsets can reach 2^32.
template <typename T>
__device__ __forceinline__ void put_at(void* out, uint64_t i, uint64_t v) {
  reinterpret_cast<T*>(out)[i] = (T)v;
}

template <int MODE, int OUT64>
__device__ __forceinline__ void phase_b(const ScanArgs& A, const Pend& p, const uint32_t (&ms)[kRows][kWave],
                                        uint64_t count, uint32_t S_w, int lane) {
  typedef typename std::conditional<OUT64 != 0, uint64_t, uint32_t>::type OutT;
  const uint64_t obase = A.obj_base - A.shift;      // object offset = obase + aligned coordinate
  const uint64_t last = A.cap - 1;
  bool ovf = false;
  if constexpr (MODE == kFasta) {
    // entering inside a line that already emitted: its first '>' is not a header, its first '\n' ends
    // the pending header of an earlier range
    bool drop = S_w && p.fV;
    const int fn_off = p.fn_off;
    const bool add_end = S_w && fn_off >= 0;
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const uint32_t mr = (p.rows >> r) & 1u ? ms[r][lane] : 0u;
      uint32_t e = mr & kOdd, n = mr & kEven;
      if (add_end && (fn_off >> 10) == r && lane == ((fn_off >> 4) & 63)) n |= 1u << (2 * (fn_off & 15));
      if (drop) {
        const uint64_t bal = __ballot(e != 0u);
        if (bal) {
          if (lane == (int)__builtin_ctzll(bal)) e &= e - 1u;
          drop = false;
        }
      }
      if (__ballot((e | n) != 0u) == 0ull) continue;
      uint32_t tot;
      const uint32_t ex = wave_excl<3>((uint32_t)__popc(e), tot);
      const uint64_t i0 = count + ex;
      const uint64_t rowb = obase + p.wbase + (uint64_t)r * kRowBytes;
      const uint64_t ob = rowb + (uint64_t)lane * 16;
      const bool near4g = !OUT64 && rowb + kRowBytes + 1 > 0xFFFFFFFFull;   // wave-uniform
      for (uint32_t x = e; x; x &= x - 1u) {
        const int bb = __builtin_ctz(x);
        const uint64_t i = i0 + (uint32_t)__popc(e & ((1u << bb) - 1u));
        const uint64_t val = ob + (uint64_t)(bb >> 1);
        if (near4g) ovf |= val > 0xFFFFFFFFull;
        put_at<OutT>(A.out, 2 * (i < last ? i : last), val);
      }
      for (uint32_t x = n; x; x &= x - 1u) {
        const int bb = __builtin_ctz(x);
        const uint64_t i = i0 + (uint32_t)__popc(e & ((1u << bb) - 1u)) - 1u;
        const uint64_t val = ob + (uint64_t)(bb >> 1) + 1u;
        if (near4g) ovf |= val > 0xFFFFFFFFull;
        put_at<OutT>(A.out, 2 * (i < last ? i : last) + 1, val);
      }
      count += tot;
    }
  } else {
    const uint32_t kk = A.every_k;
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      if (!((p.rows >> r) & 1u)) continue;
      const uint32_t mm = ms[r][lane];
      uint32_t tot;
      const uint32_t ex = wave_excl<5>((uint32_t)__popc(mm), tot);
      const uint64_t i0 = count + ex;
      const uint64_t rowb = obase + p.wbase + (uint64_t)r * kRowBytes + A.emit_add;
      const uint64_t ob = rowb + (uint64_t)lane * 16;
      const bool near4g = !OUT64 && rowb + kRowBytes > 0xFFFFFFFFull;
      if (kk == 1) {
        for (uint32_t x = mm; x; x &= x - 1u) {
          const int bb = __builtin_ctz(x);
          const uint64_t gi = i0 + (uint32_t)__popc(mm & ((1u << bb) - 1u));
          const uint64_t val = ob + (uint64_t)bb;
          if (near4g) ovf |= val > 0xFFFFFFFFull;
          put_at<OutT>(A.out, gi < last ? gi : last, val);
        }
      } else {
        for (uint32_t x = mm; x; x &= x - 1u) {
          const int bb = __builtin_ctz(x);
          uint64_t gi = i0 + (uint32_t)__popc(mm & ((1u << bb) - 1u));
          if (gi % kk != kk - 1) continue;
          gi /= kk;
          const uint64_t val = ob + (uint64_t)bb;
          if (near4g) ovf |= val > 0xFFFFFFFFull;
          put_at<OutT>(A.out, gi < last ? gi : last, val);
        }
      }
      count += tot;
    }
  }
  if (ovf) atomicOr(A.err, kErrOverflow);
}

// Bounded LDS poll for a value written by another wave of the workgroup.
__device__ __forceinline__ bool lds_wait_eq(const uint32_t* p, uint32_t v, uint32_t* err) {
  for (uint32_t spins = 0; lds_ld(p) != v; ++spins) {
    if (spins > kSpinLimit) {
      if (__lane_id() == 0) atomicOr(err, kErrTimeout);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  cbar();
  return true;
}

// !DP_STEAL: the data wave's own phase B of unit j, once the coordinator has published its prefixes.
template <int MODE, int OUT64>
__device__ __forceinline__ void data_finish(const ScanArgs& A, uint64_t j, int lane, int wave, Shared& sh PROF_ARG) {
  const int s = (int)((uint32_t)j % (uint32_t)kRing);
  PROF_MARK(2);
  lds_wait_eq(&sh.ready[s], (uint32_t)j + 1u, A.err);
  PROF_MARK(3);
  Pend p = sh.pend[s][wave];
  p.wbase = rfl64(p.wbase);
  p.rows = rfl(p.rows);
  p.fV = rfl(p.fV);
  p.fn_off = (int)rfl((uint32_t)p.fn_off);
  const uint64_t P = rfl64(sh.P[s][wave]);
  const uint32_t S = rfl(sh.S[s][wave]);
  phase_b<MODE, OUT64>(A, p, sh.m[s][wave], P, S, lane);
  PROF_MARK(4);
}

#if DP_STEAL
__device__ __forceinline__ uint32_t lds_cas(uint32_t* p, uint32_t expect, uint32_t desired) {
  __hip_atomic_compare_exchange_strong(p, &expect, desired, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
  return expect;                                     // the value seen (== old expect on success)
}

// Phase B is work-shared: task t = (unit t/15, wave t%15) needs only LDS state (masks, pend, the wave's
// prefix), so whichever data wave is free runs it.  Tasks are claimed in order, and only once their
// unit is resolved (ready).  A fast wave thus takes over the slow waves' phase B instead of idling.
template <int MODE, int OUT64>
__device__ __forceinline__ bool try_b_task(const ScanArgs& A, uint64_t K, int lane, Shared& sh PROF_ARG) {
  uint32_t t = 0, got = 0;
  if (lane == 0) {
    uint32_t cur = lds_ld(&sh.bclaim);
    for (;;) {
      const uint32_t j = cur / (uint32_t)kDataWaves;
      if ((uint64_t)j >= K || lds_ld(&sh.ready[j % (uint32_t)kRing]) != j + 1u) break;
      const uint32_t seen = lds_cas(&sh.bclaim, cur, cur + 1u);
      if (seen == cur) {
        got = 1;
        t = cur;
        break;
      }
      cur = seen;
    }
  }
  if (!rfl(got)) return false;
  t = rfl(t);
  PROF_MARK(3);
  const uint32_t j = t / (uint32_t)kDataWaves, w = t % (uint32_t)kDataWaves;
  const int s = (int)(j % (uint32_t)kRing);
  cbar();
  Pend p = sh.pend[s][w];
  p.wbase = rfl64(p.wbase);
  p.rows = rfl(p.rows);
  p.fV = rfl(p.fV);
  p.fn_off = (int)rfl((uint32_t)p.fn_off);
  const uint64_t P = rfl64(sh.P[s][w]);
  const uint32_t S = rfl(sh.S[s][w]);
  phase_b<MODE, OUT64>(A, p, sh.m[s][w], P, S, lane);
  cbar();
  if (lane == 0) lds_add(&sh.bdone[s], 1u);
  PROF_MARK(4);
  return true;
}

// Before phase A of unit k reuses its ring slot, every phase-B task of unit k - kRing must be finished;
// meanwhile, do phase-B work.  Bounded wait.
template <int MODE, int OUT64>
__device__ __forceinline__ void wait_slot(const ScanArgs& A, uint64_t k, uint64_t K, int lane, Shared& sh PROF_ARG) {
  if (k < (uint64_t)kRing) return;
  const int s = (int)((uint32_t)k % (uint32_t)kRing);
  const uint32_t target = (uint32_t)kDataWaves * (uint32_t)(k / kRing);
  for (uint32_t spins = 0; lds_ld(&sh.bdone[s]) < target;) {
    if (try_b_task<MODE, OUT64>(A, K, lane, sh PROF_PASS)) continue;
    if (++spins > kSpinLimit) {
      if (lane == 0) atomicOr(A.err, kErrTimeout);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  cbar();
}
#endif  // DP_STEAL

// The unit's 15 wave summaries composed lane-parallel: lane i < 15 holds wave i, an inclusive DPP scan over
// row 0 gives every wave's exclusive prefix function (lane i-1's inclusive) and the unit's function (lane 15,
// whose own summary is the identity).
__device__ __forceinline__ Func compose_unit(Shared& sh, int s, int lane) {
  Func w = Func{0, 0, 0, 1};
  if (lane < kDataWaves) w = Func{sh.cF[s][lane], sh.cT[s][lane], sh.sF[s][lane], sh.sT[s][lane]};
  Func inc = w;
  inc = f_then(fn_dpp<kRowShr1, 0xF>(inc), inc);
  inc = f_then(fn_dpp<kRowShr2, 0xF>(inc), inc);
  inc = f_then(fn_dpp<kRowShr4, 0xF>(inc), inc);
  inc = f_then(fn_dpp<kRowShr8, 0xF>(inc), inc);
  const Func ex = fn_dpp<kRowShr1, 0xF>(inc);
  if (lane < kDataWaves) {
    sh.exF[s][lane] = ex.cF;
    sh.exT[s][lane] = ex.cT;
    sh.esF[s][lane] = ex.sF;
    sh.esT[s][lane] = ex.sT;
  }
  const Func unit = Func{readlane64(inc.cF, kDataWaves), readlane64(inc.cT, kDataWaves),
                         (uint32_t)__builtin_amdgcn_readlane((int)inc.sF, kDataWaves),
                         (uint32_t)__builtin_amdgcn_readlane((int)inc.sT, kDataWaves)};
  if (lane == 0) {
    sh.uF[s] = unit.cF;
    sh.uT[s] = unit.cT;
    sh.usF[s] = unit.sF;
    sh.usT[s] = unit.sT;
  }
  return unit;
}

// One data-wave step with unit k: wait for its ring slot (doing phase-B tasks meanwhile) -> phase A(k) on
// buffer b -> post (the last wave composes and publishes the unit) -> prefetch the unit after next into b
// -> phase-B tasks while any are ready.
template <int MODE, int OUT64>
__device__ __forceinline__ void data_step(const ScanArgs& A, const Tab& T, uint64_t k, uint64_t K, uint64_t u0,
                                          uint64_t G,
                                          Geo& g, Geo& gnext, Buf& b, Cursor& cur, int lane, int wave, Shared& sh
                                          PROF_ARG) {
  const int s = (int)((uint32_t)k % (uint32_t)kRing);
  set_prio(((uint32_t)(wave >> 2) + (uint32_t)k) % 3u);   // 0..2: the coordinator (3) always wins
#if DP_STEAL
  PROF_MARK(2);
  wait_slot<MODE, OUT64>(A, k, K, lane, sh PROF_PASS);
  PROF_MARK(3);
#endif
  Pend p;
  const Func ws = phase_a<MODE>(A, g, b, p, sh.m[s][wave], lane, wave PROF_PASS);
  uint32_t before = 0;
  if (lane == 0) {
    sh.cF[s][wave] = ws.cF; sh.cT[s][wave] = ws.cT; sh.sF[s][wave] = ws.sF; sh.sT[s][wave] = ws.sT;
    sh.pend[s][wave] = p;
    cbar();
    before = lds_add(&sh.done[s], 1u);
  }
  // the last data wave of the unit composes it and publishes its AGG at once: publication never waits
  // behind the coordinator's look-back (a coordinator that spun would delay every higher workgroup)
  if (DP_WAVEPUB && rfl(before) == (uint32_t)kDataWaves - 1u) {
    const Func f = compose_unit(sh, s, lane);
    const uint64_t u = u0 + k * G;
    if (lane == 0) {
      if (u > 0) st_desc(&A.desc[u], pack_agg(f));
      sh.done[s] = 0;                                  // slot's counter free for unit k + kRing
      cbar();
      lds_st(&sh.composed[s], (uint32_t)k + 1u);
    }
  }
  const Geo g2 = geo_of(T, A.nchunks, A.nunits, u0 + (k + 2) * (uint64_t)G, cur);
  load_buf(b, A, g2, wave, lane);
#if DP_STEAL
  PROF_MARK(2);
  while (try_b_task<MODE, OUT64>(A, K, lane, sh PROF_PASS)) {}
#else
  if (k >= (uint64_t)kBLag) data_finish<MODE, OUT64>(A, k - kBLag, lane, wave, sh PROF_PASS);
  else PROF_MARK(2);
#endif
  g = gnext;
  gnext = g2;
}

// Coordinator: resolve unit j (look-back -> inclusive prefix, per-wave prefixes, per-chunk results) as
// soon as its data waves have composed it.
template <int MODE>
__device__ __forceinline__ void coordinator(const ScanArgs& A, const Tab& T, uint64_t u0, uint64_t G, uint64_t K,
                                            int lane, Shared& sh) {
  PROF_DECL;
  set_prio(3);
  Cursor cur{0, 0, 0, 0, 0, 0};
  uint64_t prevP = 0;
  uint32_t prevS = 0;
  uint64_t pre[4] = {0, 0, 0, 0};
  bool have_pre = false;
  uint64_t published = 0;
  (void)published;
  for (uint64_t j = 0; j < K; ++j) {
    const int s = (int)((uint32_t)j % (uint32_t)kRing);
    // by the time this workgroup has composed unit j + kLag, the lower workgroups have almost always
    // published unit j's round: resolving earlier only spins on their descriptors
    const uint64_t jw = j + kLag < K ? j + kLag : K - 1;
#if DP_WAVEPUB
    PROF_MARK(3);
    lds_wait_eq(&sh.composed[(uint32_t)jw % (uint32_t)kRing], (uint32_t)jw + 1u, A.err);
    PROF_MARK(0);
#else
    while (published <= jw) {
      const int sp = (int)((uint32_t)published % (uint32_t)kRing);
      PROF_MARK(3);
      lds_wait_eq(&sh.done[sp], (uint32_t)kDataWaves, A.err);
      PROF_MARK(0);
      const Func f = compose_unit(sh, sp, lane);
      const uint64_t up = u0 + published * G;
      if (up > 0 && lane == 0) st_desc(&A.desc[up], pack_agg(f));
      ++published;
      PROF_MARK(1);
    }
#endif
    const uint64_t u = u0 + j * G;
    const Func unit = Func{rfl64(sh.uF[s]), rfl64(sh.uT[s]), rfl(sh.usF[s]), rfl(sh.usT[s])};
    const Geo g = geo_of(T, A.nchunks, A.nunits, u, cur);
    uint64_t P;
    uint32_t S_in;
    PROF_MARK(3);
    lookback(A, u, G, u >= G ? prevP : 0ull, u >= G ? prevS : 0u, lane, P, S_in, pre, have_pre PROF_PASS);
    PROF_MARK(2);
    const uint64_t P_incl = P + (S_in ? unit.cT : unit.cF);
    const uint32_t S_out = S_in ? unit.sT : unit.sF;
    prevP = P_incl;
    prevS = S_out;
    const uint32_t st0 = g.first ? 0u : S_in;
    if (lane < kDataWaves) {                          // per-wave prefixes, one lane per wave
      sh.P[s][lane] = P + (st0 ? sh.exT[s][lane] : sh.exF[s][lane]);
      sh.S[s][lane] = st0 ? sh.esT[s][lane] : sh.esF[s][lane];
    }
    if (lane == 0) {
      st_desc(&A.desc[u], pack_prefix(P_incl, S_out));
      if (u + 1 == A.nunits) A.total[0] = P_incl;
      if (g.last) {
        A.chunk_end[g.c] = P_incl;
        if constexpr (MODE == kFasta) A.pending[g.c] = S_out ? (long long)P_incl - 1 : -1ll;
      }
    }
    // LDS ops of one wave complete in order: every lane's P/S write lands before lane 0's flag
    cbar();
    if (lane == 0) {
#if !DP_WAVEPUB
      sh.done[s] = 0;                                // slot's counter free for unit j + kRing
      cbar();
#endif
      lds_st(&sh.ready[s], (uint32_t)j + 1u);
    }
#if DP_LBPREFETCH
    // prefetch the next unit's look-back window: its latency overlaps the wait for the data waves
    have_pre = j + 1 < K;
    if (have_pre) lb_load(A, u + G, G, 0, pack_prefix(P_incl, S_out), lane, pre);
#endif
  }
  PROF_MARK(3);
  PROF_FLUSH(kCoord);
}

template <int MODE, int OUT64>
__global__ void __launch_bounds__(kThreads) scan_kernel(ScanArgs A, const uint64_t* __restrict__ tab_lo,
                                                        const uint64_t* __restrict__ tab_hi,
                                                        const uint64_t* __restrict__ tab_u0) {
  const int lane = __lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __shared__ Shared sh;
  const Tab T{(cu64*)tab_lo, (cu64*)tab_hi, (cu64*)tab_u0};
  const uint64_t G = gridDim.x;
  const uint64_t u0 = blockIdx.x;
  const uint64_t K = u0 < A.nunits ? (A.nunits - u0 + G - 1) / G : 0;   // units of this workgroup
  if (threadIdx.x < kRing) {
    sh.done[threadIdx.x] = 0;
    sh.composed[threadIdx.x] = 0;
    sh.bdone[threadIdx.x] = 0;
    sh.ready[threadIdx.x] = 0;
  }
  if (threadIdx.x == 0) sh.bclaim = 0;
  __syncthreads();
  if (wave == kCoord) {
    coordinator<MODE>(A, T, u0, G, K, lane, sh);
  } else {
    PROF_DECL;
    Cursor cur{0, 0, 0, 0, 0, 0};
    Geo g = geo_of(T, A.nchunks, A.nunits, u0, cur);
    Geo gnext = geo_of(T, A.nchunks, A.nunits, u0 + G, cur);
    Buf bA, bB;
    load_buf(bA, A, g, wave, lane);
    load_buf(bB, A, gnext, wave, lane);
    uint64_t k = 0;
    PROF_MARK(5);
    while (k < K) {
      data_step<MODE, OUT64>(A, T, k, K, u0, G, g, gnext, bA, cur, lane, wave, sh PROF_PASS);
      if (++k == K) break;
      data_step<MODE, OUT64>(A, T, k, K, u0, G, g, gnext, bB, cur, lane, wave, sh PROF_PASS);
      ++k;
    }
    drain_bufs(bA, bB);
    PROF_MARK(6);
#if !DP_STEAL
    const uint64_t j0 = K > (uint64_t)kBLag ? K - kBLag : 0;
    for (uint64_t j = j0; j < K; ++j) data_finish<MODE, OUT64>(A, j, lane, wave, sh PROF_PASS);
#else
    // drain: phase-B tasks until every task of the workgroup's K units has been claimed
    const uint32_t all = (uint32_t)kDataWaves * (uint32_t)K;
    for (uint32_t spins = 0; lds_ld(&sh.bclaim) < all;) {
      if (try_b_task<MODE, OUT64>(A, K, lane, sh PROF_PASS)) continue;
      if (++spins > kSpinLimit) {
        if (lane == 0) atomicOr(A.err, kErrTimeout);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
#endif
    PROF_MARK(6);
    PROF_FLUSH(wave);
  }
}

// first position >= from (aligned coords) holding the delimiter, inside [from, end); -1 if none.  One wave.
__device__ uint64_t wave_find(const uint8_t* base, uint64_t from, uint64_t end, uint32_t pat, int lane, bool& found) {
  for (uint64_t a = from & ~15ull; a < end; a += kRowBytes) {
    const uint64_t pa = a + (uint64_t)lane * 16;
    uint32_t m = 0;
    if (pa < end) m = mask16(*reinterpret_cast<const uint4*>(base + pa), pat) & range16((int64_t)from - (int64_t)pa, (int64_t)end - (int64_t)pa);
    const uint64_t bal = __ballot(m != 0u);
    if (bal) {
      const int l = (int)__builtin_ctzll(bal);
      const uint64_t p = pa + (m ? (uint64_t)__builtin_ctz(m) : 0ull);
      found = true;
      return readlane64(p, l);
    }
  }
  found = false;
  return 0;
}

struct ResolveArgs {
  const uint8_t* base;
  uint64_t shift, obj_base, buf_end, obj_size;   // buf_end in aligned coords
  int at_obj_end;
  const uint64_t* chunk_hi;
  uint64_t nchunks;
  long long* pending;
  void* out;
  uint64_t cap;
  int out_u64;
  uint32_t* err;
};

__global__ void __launch_bounds__(kWave) fasta_resolve_kernel(ResolveArgs R) {
  const int lane = __lane_id();
  for (uint64_t c = blockIdx.x; c < R.nchunks; c += gridDim.x) {
    const long long idx = R.pending[c];
    if (idx < 0) continue;
    bool found;
    const uint64_t p = wave_find(R.base, R.chunk_hi[c], R.buf_end, kNL, lane, found);
    uint64_t val;
    if (found) val = R.obj_base - R.shift + p + 1;
    else if (R.at_obj_end) val = R.obj_size;
    else continue;   // unresolved: the host extends the buffer
    if (lane == 0) {
      if ((uint64_t)idx < R.cap) {
        if (R.out_u64) put<uint64_t>(R.out, 2 * (uint64_t)idx + 1, val);
        else {
          if (val > 0xFFFFFFFFull) atomicOr(R.err, kErrOverflow);
          put<uint32_t>(R.out, 2 * (uint64_t)idx + 1, val);
        }
      }
      R.pending[c] = -1;
    }
  }
}

__global__ void __launch_bounds__(kWave) find_kernel(const uint8_t* base, uint64_t from, uint64_t end, uint32_t pat,
                                                    long long* res) {
  bool found;
  const uint64_t p = wave_find(base, from, end, pat, __lane_id(), found);
  if (__lane_id() == 0) *res = found ? (long long)p : -1ll;
}

// ------------------------------------------------------------------------------------------ calibration
// Plain read-only stream (16 B per lane, grid-stride, 4 loads in flight per lane): the achievable HBM
// read rate on this device, reported next to the scan's roofline fraction.
__global__ void __launch_bounds__(256) stream_read_kernel(const uint4* __restrict__ p, uint64_t n16,
                                                         unsigned* __restrict__ sink) {
  uint32_t acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
  }
  for (; i < n16; i += stride) {
    const uint4 a = p[i];
    acc ^= a.x ^ a.y ^ a.z ^ a.w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;   // keeps the loads alive; practically never stores
}

// ------------------------------------------------------------------------------------------ host side
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(expr)                                                                       \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      return fail(DP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));          \
  } while (0)

}  // namespace

struct dp_ctx {
  int device = 0;
  hipStream_t own = nullptr, stream = nullptr;
  int cus = 0;
  int grid = 0;                       // persistent scan grid
  // device workspace
  unsigned long long* d_desc = nullptr;
  uint64_t desc_cap = 0;
  uint64_t* d_tab = nullptr;          // chunk_lo | chunk_hi | chunk_u0 | pending | ctrl
  uint64_t tab_cap = 0;               // in u64 words
  uint64_t* h_tab = nullptr;          // pinned mirror
  uint64_t h_cap = 0;
  std::vector<uint64_t> last_tab;     // last uploaded table (skip identical re-uploads)
  uint64_t* d_tab_uploaded = nullptr;
  // async call state
  int inflight = -1;                  // -1 none, kFasta, kDelim, 9 find
  uint64_t nchunks = 0, cap = 0;
  int out_u64 = 0;
  uint32_t every_k = 1;
  uint64_t pend_off = 0, ctrl_off = 0;
  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  double ms_acc = 0.0;
  uint64_t launches = 0;
};

namespace {

int ensure_tab(dp_ctx* c, uint64_t words) {
  if (words > c->tab_cap) {
    if (c->d_tab) HIPCHK(hipFree(c->d_tab));
    uint64_t cap = words + words / 2 + 64;
    HIPCHK(hipMalloc(&c->d_tab, cap * 8));
    c->tab_cap = cap;
    c->last_tab.clear();
  }
  if (words > c->h_cap) {
    if (c->h_tab) HIPCHK(hipHostFree(c->h_tab));
    uint64_t cap = words + words / 2 + 64;
    HIPCHK(hipHostMalloc(&c->h_tab, cap * 8, hipHostMallocDefault));
    c->h_cap = cap;
  }
  return DP_OK;
}
int ensure_desc(dp_ctx* c, uint64_t n) {
  if (n > c->desc_cap) {
    if (c->d_desc) HIPCHK(hipFree(c->d_desc));
    uint64_t cap = ((n + n / 4 + 1023) / 1024) * 1024;
    HIPCHK(hipMalloc(&c->d_desc, cap * 8));
    c->desc_cap = cap;
  }
  return DP_OK;
}
int ev_begin(dp_ctx* c, hipEvent_t* e0) {
  if (!c->timing) return DP_OK;
  while (c->ev_pool.size() < c->ev_used + 2) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    c->ev_pool.push_back(e);
  }
  *e0 = c->ev_pool[c->ev_used];
  HIPCHK(hipEventRecord(*e0, c->stream));
  return DP_OK;
}
int ev_end(dp_ctx* c) {
  if (!c->timing) return DP_OK;
  HIPCHK(hipEventRecord(c->ev_pool[c->ev_used + 1], c->stream));
  c->ev_used += 2;
  return DP_OK;
}
int harvest_events(dp_ctx* c) {
  for (size_t i = 0; i + 1 < c->ev_used; i += 2) {
    HIPCHK(hipEventSynchronize(c->ev_pool[i + 1]));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, c->ev_pool[i], c->ev_pool[i + 1]));
    c->ms_acc += ms;
    c->launches += 1;
  }
  c->ev_used = 0;
  return DP_OK;
}

// Lay out the chunk table in aligned coordinates and enqueue its upload + the control-block reset.
// Table layout (u64 words): lo[n] hi[n] u0[n+1] pending[n] chunk_end[n] ctrl[4] (err | total | spare x2).
int stage_chunks(dp_ctx* c, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base, const uint64_t* chunks,
                 uint64_t n, uint64_t* nunits_out) {
  const uint64_t shift = (uint64_t)((uintptr_t)d_buf & 15u);
  std::vector<uint64_t> tab(3 * n + 1);
  uint64_t units = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t c0 = chunks[2 * i], c1 = chunks[2 * i + 1];
    if (c1 < c0 || c0 < buf_base || c1 > buf_base + buf_len)
      return fail(DP_ERR_INVALID, "chunk " + std::to_string(i) + " [" + std::to_string(c0) + "," +
                                      std::to_string(c1) + ") outside the buffer");
    const uint64_t lo = c0 - buf_base + shift, hi = c1 - buf_base + shift;
    tab[i] = lo;
    tab[n + i] = hi;
    tab[2 * n + i] = units;
    if (hi > lo) units += (hi - (lo & ~15ull) + kUnitBytes - 1) / kUnitBytes;
  }
  tab[3 * n] = units;
  const uint64_t words = 5 * n + 1 + 4;
  int rc = ensure_tab(c, words);
  if (rc) return rc;
  c->pend_off = 3 * n + 1;
  c->ctrl_off = 5 * n + 1;
  if (tab != c->last_tab) {
    // the pinned mirror may still feed an earlier async copy: wait for the stream before rewriting it
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(c->h_tab, tab.data(), tab.size() * 8);
    HIPCHK(hipMemcpyAsync(c->d_tab, c->h_tab, tab.size() * 8, hipMemcpyHostToDevice, c->stream));
    c->last_tab.swap(tab);
  }
  HIPCHK(hipMemsetAsync(c->d_tab + c->pend_off, 0xFF, 2 * n * 8, c->stream));
  HIPCHK(hipMemsetAsync(c->d_tab + c->ctrl_off, 0, 4 * 8, c->stream));
  *nunits_out = units;
  return DP_OK;
}

int launch_scan(dp_ctx* c, int mode, const uint8_t* d_buf, uint64_t buf_base, uint64_t n, uint64_t units,
                void* d_out, int out_u64, uint64_t cap, uint32_t delim, uint32_t every_k, uint32_t emit_add) {
  const uint64_t shift = (uint64_t)((uintptr_t)d_buf & 15u);
  ScanArgs a;
  a.base = d_buf - shift;
  a.shift = shift;
  a.obj_base = buf_base;
  a.nchunks = n;
  a.nunits = units;
  a.desc = c->d_desc;
  if (cap == 0 || d_out == nullptr) {                 // count-only call: stores go to a scratch slot
    d_out = c->d_tab + c->ctrl_off + 2;                // ctrl spare words (16 B)
    cap = 1;
  }
  a.out = d_out;
  a.cap = cap;
  a.out_u64 = out_u64;
  a.delim = delim * 0x01010101u;
  a.every_k = every_k;
  a.emit_add = emit_add;
  a.err = reinterpret_cast<uint32_t*>(c->d_tab + c->ctrl_off);
  a.total = reinterpret_cast<unsigned long long*>(c->d_tab + c->ctrl_off + 1);
  a.pending = reinterpret_cast<long long*>(c->d_tab + c->pend_off);
  a.chunk_end = reinterpret_cast<unsigned long long*>(c->d_tab + c->pend_off + n);
  if (units == 0) return DP_OK;
  int rc = ensure_desc(c, units);
  if (rc) return rc;
  a.desc = c->d_desc;
  HIPCHK(hipMemsetAsync(c->d_desc, 0, ((units * 8 + 15) / 16) * 16, c->stream));
  const unsigned grid = (unsigned)(units < (uint64_t)c->grid ? units : (uint64_t)c->grid);
  hipEvent_t e0;
  rc = ev_begin(c, &e0);
  if (rc) return rc;
  const uint64_t* tlo = c->d_tab;
  const uint64_t* thi = c->d_tab + n;
  const uint64_t* tu0 = c->d_tab + 2 * n;
  if (mode == kFasta && !out_u64)
    hipLaunchKernelGGL((scan_kernel<kFasta, 0>), dim3(grid), dim3(kThreads), 0, c->stream, a, tlo, thi, tu0);
  else if (mode == kFasta)
    hipLaunchKernelGGL((scan_kernel<kFasta, 1>), dim3(grid), dim3(kThreads), 0, c->stream, a, tlo, thi, tu0);
  else if (!out_u64)
    hipLaunchKernelGGL((scan_kernel<kDelim, 0>), dim3(grid), dim3(kThreads), 0, c->stream, a, tlo, thi, tu0);
  else
    hipLaunchKernelGGL((scan_kernel<kDelim, 1>), dim3(grid), dim3(kThreads), 0, c->stream, a, tlo, thi, tu0);
  HIPCHK(hipGetLastError());
  return ev_end(c);
}

int check_ctx(dp_ctx* c) {
  if (!c) return fail(DP_ERR_INVALID, "null dp_ctx");
  HIPCHK(hipSetDevice(c->device));
  return DP_OK;
}

int collect_ctrl(dp_ctx* c, uint64_t extra_words) {
  // D2H of [pending (nchunks) | ctrl(4)] and wait
  const uint64_t off = c->pend_off;
  const uint64_t words = c->ctrl_off + 4 - off + extra_words;
  HIPCHK(hipMemcpyAsync(c->h_tab + off, c->d_tab + off, words * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  int rc = harvest_events(c);
  if (rc) return rc;
  return DP_OK;
}

}  // namespace

extern "C" {

int dp_abi_version(void) { return 1; }

const char* dp_last_error(void) { return g_err.c_str(); }

int dp_device_count(int* n) {
  if (!n) return fail(DP_ERR_INVALID, "null");
  HIPCHK(hipGetDeviceCount(n));
  return DP_OK;
}

int dp_ctx_create(int device, dp_ctx** out) {
  if (!out) return fail(DP_ERR_INVALID, "null out");
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(DP_ERR_INVALID, "device " + std::to_string(device) + " out of range");
  HIPCHK(hipSetDevice(device));
  dp_ctx* c = new dp_ctx();
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return fail(DP_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  c->stream = c->own;
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  c->cus = prop.multiProcessorCount;
  int occ = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (scan_kernel<kFasta, 0>), kThreads, 0));
  const void* others[] = {(const void*)scan_kernel<kFasta, 1>, (const void*)scan_kernel<kDelim, 0>,
                          (const void*)scan_kernel<kDelim, 1>};
  for (const void* k : others) {
    int o = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k, kThreads, 0));
    if (o < occ) occ = o;
  }
  // every workgroup of the persistent grid must be resident (look-back waits on lower units): stay one
  // block per CU under the occupancy answer (it can over-report by one, MI355X_MICROARCH.md §Residency)
  // one workgroup (8 waves) per CU: the look-back window is the grid, so G <= 256 keeps it one load
  int per_cu = 1;
  const char* env = getenv("DP_BLOCKS_PER_CU");
  if (env) per_cu = atoi(env);
  if (per_cu > occ - 1) per_cu = occ - 1;
  if (per_cu < 1) per_cu = 1;
  c->grid = c->cus * per_cu;
  *out = c;
  return DP_OK;
}

int dp_ctx_destroy(dp_ctx* c) {
  if (!c) return DP_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto e : c->ev_pool) (void)hipEventDestroy(e);
  if (c->d_desc) (void)hipFree(c->d_desc);
  if (c->d_tab) (void)hipFree(c->d_tab);
  if (c->h_tab) (void)hipHostFree(c->h_tab);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
  return DP_OK;
}

int dp_ctx_get_stream(dp_ctx* c, void** s) {
  if (!c || !s) return fail(DP_ERR_INVALID, "null");
  *s = (void*)c->stream;
  return DP_OK;
}

int dp_ctx_set_stream(dp_ctx* c, void* s) {
  if (!c) return fail(DP_ERR_INVALID, "null");
  c->stream = s ? (hipStream_t)s : c->own;
  return DP_OK;
}

int dp_ctx_device(dp_ctx* c, int* d) {
  if (!c || !d) return fail(DP_ERR_INVALID, "null");
  *d = c->device;
  return DP_OK;
}

int dp_malloc(dp_ctx* c, uint64_t bytes, void** p) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (!p) return fail(DP_ERR_INVALID, "null");
  HIPCHK(hipMalloc(p, bytes ? bytes : 16));
  return DP_OK;
}

int dp_free(dp_ctx* c, void* p) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (p) HIPCHK(hipFree(p));
  return DP_OK;
}

int dp_host_alloc(uint64_t bytes, void** p) {
  if (!p) return fail(DP_ERR_INVALID, "null");
  HIPCHK(hipHostMalloc(p, bytes ? bytes : 16, hipHostMallocDefault));
  return DP_OK;
}

int dp_host_free(void* p) {
  if (p) HIPCHK(hipHostFree(p));
  return DP_OK;
}

int dp_h2d(dp_ctx* c, void* dst, const void* src, uint64_t n) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (n) HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c->stream));
  return DP_OK;
}

int dp_d2h(dp_ctx* c, void* dst, const void* src, uint64_t n) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (n) HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->stream));
  return DP_OK;
}

int dp_sync(dp_ctx* c) {
  int rc = check_ctx(c);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(c->stream));
  return DP_OK;
}

int dp_fasta_index_async(dp_ctx* c, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base, uint64_t obj_size,
                         const uint64_t* chunks, uint64_t nchunks, void* d_out, int out_u64, uint64_t cap_pairs) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (c->inflight >= 0) return fail(DP_ERR_INVALID, "a scan is already in flight on this ctx");
  if (nchunks && (!d_buf || !chunks)) return fail(DP_ERR_INVALID, "null buffer/chunks");
  if (cap_pairs && !d_out) return fail(DP_ERR_INVALID, "null output with cap > 0");
  if (buf_base + buf_len > obj_size) return fail(DP_ERR_INVALID, "buffer extends beyond the object");
  uint64_t units = 0;
  rc = stage_chunks(c, d_buf, buf_len, buf_base, chunks, nchunks, &units);
  if (rc) return rc;
  rc = launch_scan(c, kFasta, d_buf, buf_base, nchunks, units, d_out, out_u64, cap_pairs, 0, 1, 0);
  if (rc) return rc;
  if (nchunks) {
    const uint64_t shift = (uint64_t)((uintptr_t)d_buf & 15u);
    ResolveArgs r;
    r.base = d_buf - shift;
    r.shift = shift;
    r.obj_base = buf_base;
    r.buf_end = shift + buf_len;
    r.obj_size = obj_size;
    r.at_obj_end = (buf_base + buf_len == obj_size);
    r.chunk_hi = c->d_tab + nchunks;
    r.nchunks = nchunks;
    r.pending = reinterpret_cast<long long*>(c->d_tab + c->pend_off);
    r.out = d_out;
    r.cap = cap_pairs;
    r.out_u64 = out_u64;
    r.err = reinterpret_cast<uint32_t*>(c->d_tab + c->ctrl_off);
    const unsigned g = (unsigned)(nchunks < 4096 ? nchunks : 4096);
    hipLaunchKernelGGL(fasta_resolve_kernel, dim3(g), dim3(kWave), 0, c->stream, r);
    HIPCHK(hipGetLastError());
  }
  c->inflight = kFasta;
  c->nchunks = nchunks;
  c->cap = cap_pairs;
  c->out_u64 = out_u64;
  return DP_OK;
}

int dp_fasta_result(dp_ctx* c, uint64_t* n_pairs, int64_t* pending, uint64_t* chunk_end) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (c->inflight != kFasta) return fail(DP_ERR_INVALID, "no FASTA scan in flight on this ctx");
  c->inflight = -1;
  rc = collect_ctrl(c, 0);
  if (rc) return rc;
  const uint32_t err = (uint32_t)c->h_tab[c->ctrl_off];
  const uint64_t total = c->nchunks ? c->h_tab[c->ctrl_off + 1] : 0;
  if (n_pairs) *n_pairs = total;
  if (pending) memcpy(pending, c->h_tab + c->pend_off, c->nchunks * 8);
  if (chunk_end) {
    // empty chunks were never visited: carry the previous chunk's end
    uint64_t prev = 0;
    for (uint64_t i = 0; i < c->nchunks; ++i) {
      uint64_t e = c->h_tab[c->pend_off + c->nchunks + i];
      if (e == ~0ull) e = prev;
      chunk_end[i] = e;
      prev = e;
    }
  }
  if (err & kErrTimeout) return fail(DP_ERR_TIMEOUT, "look-back wait timed out (grid not co-resident?)");
  if (err & kErrOverflow) return fail(DP_ERR_OVERFLOW, "Python integer out of bounds for uint32");
  if (total > c->cap) return fail(DP_ERR_CAPACITY, "output capacity " + std::to_string(c->cap) + " < " +
                                                       std::to_string(total) + " pairs");
  return DP_OK;
}

int dp_fasta_index(dp_ctx* c, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base, uint64_t obj_size,
                   const uint64_t* chunks, uint64_t nchunks, void* d_out, int out_u64, uint64_t cap_pairs,
                   uint64_t* n_pairs, int64_t* pending, uint64_t* chunk_end) {
  int rc = dp_fasta_index_async(c, d_buf, buf_len, buf_base, obj_size, chunks, nchunks, d_out, out_u64, cap_pairs);
  if (rc) return rc;
  return dp_fasta_result(c, n_pairs, pending, chunk_end);
}

int dp_delim_index_async(dp_ctx* c, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base, uint64_t begin,
                         uint64_t end, uint32_t delim, uint32_t every_k, uint32_t emit_add, void* d_out,
                         int out_u64, uint64_t cap) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (c->inflight >= 0) return fail(DP_ERR_INVALID, "a scan is already in flight on this ctx");
  if (every_k == 0) return fail(DP_ERR_INVALID, "every_k must be >= 1");
  if (delim > 255) return fail(DP_ERR_INVALID, "delim must be a byte");
  if (end > begin && !d_buf) return fail(DP_ERR_INVALID, "null buffer");
  if (cap && !d_out) return fail(DP_ERR_INVALID, "null output with cap > 0");
  const uint64_t ch[2] = {begin, end};
  uint64_t units = 0;
  rc = stage_chunks(c, d_buf, buf_len, buf_base, ch, 1, &units);
  if (rc) return rc;
  rc = launch_scan(c, kDelim, d_buf, buf_base, 1, units, d_out, out_u64, cap, delim, every_k, emit_add);
  if (rc) return rc;
  c->inflight = kDelim;
  c->nchunks = 1;
  c->cap = cap;
  c->out_u64 = out_u64;
  c->every_k = every_k;
  return DP_OK;
}

int dp_delim_result(dp_ctx* c, uint64_t* n_out, uint64_t* n_delims) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (c->inflight != kDelim) return fail(DP_ERR_INVALID, "no delimiter scan in flight on this ctx");
  const uint64_t k = c->every_k;
  c->inflight = -1;
  rc = collect_ctrl(c, 0);
  if (rc) return rc;
  const uint32_t err = (uint32_t)c->h_tab[c->ctrl_off];
  const uint64_t nd = c->h_tab[c->ctrl_off + 1];
  const uint64_t nout = k ? nd / k : 0;
  if (n_delims) *n_delims = nd;
  if (n_out) *n_out = nout;
  if (err & kErrTimeout) return fail(DP_ERR_TIMEOUT, "look-back wait timed out (grid not co-resident?)");
  if (err & kErrOverflow) return fail(DP_ERR_OVERFLOW, "Python integer out of bounds for uint32");
  if (nout > c->cap) return fail(DP_ERR_CAPACITY, "output capacity " + std::to_string(c->cap) + " < " +
                                                      std::to_string(nout) + " offsets");
  return DP_OK;
}

int dp_delim_index(dp_ctx* c, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base, uint64_t begin, uint64_t end,
                   uint32_t delim, uint32_t every_k, uint32_t emit_add, void* d_out, int out_u64, uint64_t cap,
                   uint64_t* n_out, uint64_t* n_delims) {
  int rc = dp_delim_index_async(c, d_buf, buf_len, buf_base, begin, end, delim, every_k, emit_add, d_out, out_u64, cap);
  if (rc) return rc;
  return dp_delim_result(c, n_out, n_delims);
}

int dp_find_delim(dp_ctx* c, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base, uint64_t from, uint32_t delim,
                  int64_t* pos) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (!pos) return fail(DP_ERR_INVALID, "null pos");
  if (c->inflight >= 0) return fail(DP_ERR_INVALID, "a scan is already in flight on this ctx");
  if (delim > 255) return fail(DP_ERR_INVALID, "delim must be a byte");
  if (from < buf_base) return fail(DP_ERR_INVALID, "from < buffer base");
  *pos = -1;
  if (from >= buf_base + buf_len) return DP_OK;
  rc = ensure_tab(c, 8);
  if (rc) return rc;
  const uint64_t shift = (uint64_t)((uintptr_t)d_buf & 15u);
  long long* d_res = reinterpret_cast<long long*>(c->d_tab);
  c->last_tab.clear();   // the table area is reused as scratch here
  hipLaunchKernelGGL(find_kernel, dim3(1), dim3(kWave), 0, c->stream, d_buf - shift, from - buf_base + shift,
                     shift + buf_len, delim * 0x01010101u, d_res);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(c->h_tab, c->d_tab, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  const long long r = (long long)c->h_tab[0];
  *pos = r < 0 ? -1 : (int64_t)(r - (long long)shift + (long long)buf_base);
  return DP_OK;
}

int dp_stream_read(dp_ctx* c, const void* d_buf, uint64_t bytes, int blocks_per_cu) {
  int rc = check_ctx(c);
  if (rc) return rc;
  rc = ensure_tab(c, 8);
  if (rc) return rc;
  const int bpc = blocks_per_cu > 0 ? blocks_per_cu : 8;
  hipEvent_t e0;
  rc = ev_begin(c, &e0);
  if (rc) return rc;
  hipLaunchKernelGGL(stream_read_kernel, dim3((unsigned)(c->cus * bpc)), dim3(256), 0, c->stream,
                     reinterpret_cast<const uint4*>(d_buf), bytes / 16, reinterpret_cast<unsigned*>(c->d_tab));
  HIPCHK(hipGetLastError());
  return ev_end(c);
}

int dp_timing_enable(dp_ctx* c, int enable) {
  if (!c) return fail(DP_ERR_INVALID, "null");
  c->timing = enable != 0;
  return DP_OK;
}

int dp_timing_read(dp_ctx* c, double* total_ms, uint64_t* launches) {
  int rc = check_ctx(c);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(c->stream));
  rc = harvest_events(c);
  if (rc) return rc;
  if (total_ms) *total_ms = c->ms_acc;
  if (launches) *launches = c->launches;
  c->ms_acc = 0.0;
  c->launches = 0;
  return DP_OK;
}

int dp_debug_profile(dp_ctx* c, uint64_t* host_words, uint64_t n_words, int* slots, int* waves) {
#ifdef DP_PROF
  if (!c || !host_words) return fail(DP_ERR_INVALID, "dp_debug_profile: null argument");
  const uint64_t n = n_words < (uint64_t)kProfMaxGrid * kProfWaves * kProfSlots ? n_words
                                                                                 : (uint64_t)kProfMaxGrid * kProfWaves * kProfSlots;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpyFromSymbol(host_words, HIP_SYMBOL(g_prof), n * 8, 0, hipMemcpyDeviceToHost));
  if (slots) *slots = kProfSlots;
  if (waves) *waves = kProfWaves;
  return DP_OK;
#else
  (void)c; (void)host_words; (void)n_words; (void)slots; (void)waves;
  return fail(DP_ERR_INVALID, "dp_debug_profile: library built without -DDP_PROF");
#endif
}

int dp_scan_geometry(dp_ctx* c, int* grid, int* unit_bytes) {
  if (!c) return fail(DP_ERR_INVALID, "null");
  if (grid) *grid = c->grid;
  if (unit_bytes) *unit_bytes = kUnitBytes;
  return DP_OK;
}

}  // extern "C"
