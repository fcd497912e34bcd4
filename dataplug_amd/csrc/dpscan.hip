// dpscan.hip — MI355X (gfx950, CDNA4) record-boundary scan kernels + the C ABI of libdpscan.so.
//
// What ships (every kernel memory-bound integer byte work, no MFMA):
//   * FASTA header index (dataplug/formats/genomics/fasta.py:24-63 for a whole chunk plan, bit-exact):
//     map_kernel (one 16-wave workgroup per CU streams groups of 16 ranges of 16 KiB claimed from a ticket, a
//     barrier per step; per range a 16-byte summary of its header count / line state as a function of the
//     incoming state, and its events, under "no header pending", burst-stored from LDS) + fasta_place_kernel
//     (blocks of 1024 range summaries: scan, decoupled look-back over block descriptors, the pending-header
//     fix-up, LDS-staged coalesced output runs), then fasta_resolve_kernel (header ends cut by a chunk end).
//   * newline index (CSV / VCF lines, FASTQ read ends with every_k = 4): line_kernel (the map kernel's streaming
//     loop with the positions kept in LDS, a per-group decoupled look-back by LDS-DMA windows and in-kernel
//     placement) up to 4 GiB per launch and for CSV-dense input above; the one-pass look-back scan_kernel<DELIM>
//     (persistent grid, 15 data waves + a coordinator wave per workgroup, 240 KiB units) for sparser input above
//     4 GiB, picked per launch on the device by density_probe_kernel from the launch's own bytes.
//   * find_kernel (dp_find_delim), and the calibration stream kernels.
// Shared pieces: bounds-checked non-temporal buffer loads hand-waited with explicit s_waitcnt (checked by the
// ISA guard, dataplug_amd/isa_guard.py, before a build is installed); byte classes by v_perm_b32 with all-ones
// sources (perm(-1, -1, w ^ (pattern ^ 0x0C0C0C0C)) flags the pattern bytes exactly, 2 VALU per dword) packed
// by v_dot4_i32_i8; look-back descriptors tagged with a launch epoch (no per-launch reset); every inter-workgroup
// wait bounded in time (DP_ERR_TIMEOUT); work that waits on other workgroups claimed from tickets by running
// workgroups only, so no grid assumes co-residency.  scan_kernel<FASTA> (the one-pass FASTA form) stays for
// A/B runs (dp_ctx_set_form).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/dpscan.h"

namespace {

// The shipped geometry and policies (the variants measured against them are in DESIGN.md §4 and git history;
// round 5 removed their switches: the library is one build).
constexpr int kWave = 64;
constexpr int kDataWaves = 15;                     // + 1 coordinator wave (one-pass kernel)
static_assert(kDataWaves >= 2 && kDataWaves <= 15, "data waves: one DPP row of summaries");
constexpr int kCoord = kDataWaves;
constexpr int kWaves = kDataWaves + 1;
constexpr int kThreads = kWave * kWaves;           // 1024
constexpr int kRowBytes = kWave * 16;              // one dwordx4 per lane
constexpr int kRangeRows = 16;                     // rows per wave range
static_assert(kRangeRows * 1024 + 64 < 65536, "event positions are 16-bit offsets into a range");
constexpr int kBufs = 2;                           // input buffers per wave range: one scanned, one in flight
constexpr int kRows = kRangeRows / kBufs;          // rows per buffer (one load batch)
constexpr int kBufBytes = kRowBytes * kRows;
constexpr int kWaveBytes = kRowBytes * kRangeRows;   // 16 KiB wave range per unit
constexpr int kUnitBytes = kWaveBytes * kDataWaves;  // 240 KiB look-back unit
static_assert(kRows * kBufs == kRangeRows && kRows >= 2 && kRows <= 8, "buffers of 2, 4 or 8 rows");
// In-flight load destinations live in VGPRs (4 per 16-byte row). 1024-lane workgroups have 128 VGPRs per
// lane; past 64 of them in buffers the compiler spills live destinations to scratch, and a spilled
// un-waited destination corrupts addresses (32-row ranges in 4 buffers = 128 VGPRs faulted the GPU in round 3).
static_assert(kBufs * kRows * 4 <= 64, "input buffers must leave room in the 128-VGPR budget");
constexpr uint32_t kRing = 16;                     // unit slots per workgroup (units in flight)
// Units are claimed dynamically (a global ticket, by the coordinator, kClaimAhead steps ahead of the
// workgroup's front data wave): a workgroup only ever claims a unit while it runs, so every unit a wait
// depends on belongs to a running (or finished) workgroup — no co-residency assumption, and faster CUs
// take more units.  The queue spans the ring plus the claim-ahead distance.
constexpr uint32_t kClaimFasta = 4;                // FASTA units per claim
constexpr uint32_t kClaimDelimDense = 2;           // DELIM units per claim once a unit holds more than kClaimDense
constexpr uint32_t kClaimDelimSparse = 4;          // ... and while they hold fewer
constexpr uint32_t kClaimDense = 5500;
constexpr uint32_t kClaimAhead = 3;
constexpr uint32_t kUnitQ = 2 * kRing;
static_assert(kUnitQ >= kRing + kClaimAhead + 2, "unit queue: ring + claim-ahead");
constexpr uint32_t kEvCap = 4096;                  // 16-bit event entries per data wave (circular)
constexpr uint32_t kEvMask = kEvCap - 1;
constexpr uint32_t kDenseMax = 1024;               // events kept per wave range; more = dense
static_assert((kEvCap & kEvMask) == 0 && kEvCap >= 2 * kDenseMax, "event list: power of two, >= 2 ranges");
static_assert((kRing & (kRing - 1)) == 0 && kRing >= 2, "ring: power of two");

constexpr uint32_t kSel12 = 0x0C0C0C0Cu;           // v_perm selector that yields 0x00
constexpr uint32_t kKeyGT = 0x3E3E3E3Eu ^ kSel12;  // '>'
constexpr uint32_t kKeyNL = 0x0A0A0A0Au ^ kSel12;  // '\n'

constexpr uint32_t kErrTimeout = 1u;
constexpr uint32_t kErrOverflow = 2u;

constexpr uint64_t kStatAgg = 1ull << 62;
constexpr uint64_t kStatPrefix = 2ull << 62;
constexpr uint64_t kStatMask = 3ull << 62;
// Launch epoch in bits 50..61 of every stored descriptor (AGG uses bits 0..49, PREFIX 0..48): a descriptor
// left by an earlier launch carries another epoch and reads as "not published".  The host zeroes the
// array only when it is (re)allocated and once every kEpochMax launches.
constexpr int kEpochShift = 50;
constexpr uint64_t kEpochMask = 0xFFFull << kEpochShift;
constexpr uint32_t kEpochMax = 0xFFFu;
// Every inter-wave / inter-workgroup wait is bounded in TIME (the 100 MHz realtime counter, read every 256
// polls), not in polls: a scan may share the device with other work (a blit kernel of another thread's
// pageable copy, another process's kernels) that delays part of the grid by far more than any poll count
// would allow, while a grid that really cannot become resident must still end.
constexpr uint64_t kWaitTicks = 100000000ull * 20;   // 20 s
constexpr uint32_t kPollCheck = 255u;                // check the clock every 256 polls
__device__ __forceinline__ bool wait_expired(uint32_t spins, uint64_t& t0) {
  if ((spins & kPollCheck) != kPollCheck) return false;
  const uint64_t t = __builtin_amdgcn_s_memrealtime();
  if (t0 == 0) {
    t0 = t;
    return false;
  }
  return t - t0 > kWaitTicks;
}

enum Mode { kFasta = 0, kDelim = 1 };
// newline kernels (the codes of dp_scan_delim_form / dp_last_delim_form): lockstep line_kernel, map + placement, one-pass
constexpr uint32_t kFormLine = 1, kFormOne = 3;   // (2: round 3's map + placement newline form, removed in round 5)

// Diagnostics build only (-DDP_DIAG; dataplug_amd.build never sets it for the shipped library): realtime stamps
// (100 MHz) of the two-kernel FASTA form (map_kernel per wave, fasta_place_kernel per block) and line_kernel's
// per-step timeline, read back with dp_debug_profile() (tools/map_timeline.py, place_timeline.py,
// line_timeline.py).
#ifdef DP_DIAG
constexpr int kProfSlots = 8;
constexpr int kProfWaves = 16;
constexpr int kProfMaxGrid = 1024;
// line_kernel timeline past the per-wave slots: [256 workgroups][64 steps][waves 0, 1, 8, 15][8 events]
constexpr uint64_t kLtlBase = (uint64_t)kProfMaxGrid * kProfWaves * kProfSlots;
constexpr uint32_t kLtlSteps = 64, kLtlWaves = 4;
constexpr uint64_t kProfWords = kLtlBase + 256ull * kLtlSteps * kLtlWaves * 8;
__device__ unsigned long long g_prof[kProfWords];
#endif

struct ScanArgs {
  const uint8_t* base;         // 16-byte aligned base; coordinates below are relative to it
  uint64_t shift;              // buffer start - base (0..15)
  uint64_t obj_base;           // object offset of buffer byte 0
  uint64_t nchunks;
  uint64_t nunits;
  unsigned long long* desc;    // [nunits] look-back descriptors, tagged with the launch epoch (no per-launch reset)
  uint64_t epoch;              // this launch's tag, already at kEpochShift
  void* out;
  uint64_t cap;                // entries (FASTA: pairs)
  int out_u64;
  uint32_t wrap32;             // DELIM uint32 output as low words (paged index): no overflow check
  unsigned long long* blocktab;  // DELIM uint16 / uint8 output: entries before each 64 KiB boundary (index - tab_j0)
  uint64_t tab_j0, tab_n;
  uint16_t* subtab;            // DELIM uint8 output: low 16 bits of the entries before each 256-byte boundary
  uint64_t sub_s0, sub_n;      // (index - sub_s0)
  uint64_t carry;              // DELIM: delimiters before this launch's first byte (a streamed object's pieces)
  uint32_t delim;              // DELIM: byte replicated x4
  uint32_t every_k;
  uint32_t emit_add;
  uint32_t* err;
  unsigned long long* total;   // inclusive count at the last unit
  unsigned int* ticket;        // [2]: next unit to claim, workgroups finished (both reset by the last one)
  long long* pending;          // FASTA: [nchunks] pair index whose end is unresolved at chunk end, or -1
  unsigned long long* chunk_end;  // [nchunks] inclusive count at the end of each (non-empty) chunk
  const uint32_t* pick;        // (auto newline form) the density probe's choice: the one-pass kernel runs only if kFormOne
};

// ------------------------------------------------------------------------------------------ helpers
// 0x00 in every byte of w that equals the key's pattern byte, 0xFF in every other byte (exact).
__device__ __forceinline__ uint32_t match4(uint32_t w, uint32_t key) {
  return __builtin_amdgcn_perm(0xFFFFFFFFu, 0xFFFFFFFFu, w ^ key);
}
// match4 bytes (0x00 = 0, 0xFF = -1 as i8) of a lane's 4 dwords -> 16-bit mask, bit i = byte i matched.
// v_dot4_i32_i8 with weights 1, 2, 4, 8 subtracts the non-matching weights of one dword from its
// accumulator; combined as four independent dot4s (no accumulator chain: the dependent v_dot4c form needs
// s_nop 2 per link) by two-level shift-adds, d0 carrying the +0xFFFF: 4 dot4 + 3 shifts + 2 adds.
// DELIM output stores carry the non-temporal hint (the index is not re-read by the kernel; same-box A/B: CSV/VCF
// +2%; on FASTA's sparse 4-byte stores it measured -1 to -2%, so FASTA keeps plain stores).
typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack16(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3) {
  const int d0 = __builtin_amdgcn_sdot4((int)p0, 0x08040201, 0xFFFF, false);
  const int d1 = __builtin_amdgcn_sdot4((int)p1, 0x08040201, 0, false);
  const int d2 = __builtin_amdgcn_sdot4((int)p2, 0x08040201, 0, false);
  const int d3 = __builtin_amdgcn_sdot4((int)p3, 0x08040201, 0, false);
  const uint32_t lo = ((uint32_t)d1 << 4) + (uint32_t)d0;
  const uint32_t hi = ((uint32_t)d3 << 4) + (uint32_t)d2;
  return (hi << 8) + lo;
}
__device__ __forceinline__ uint32_t mask16(const uint4& v, uint32_t key) {
  return pack16(match4(v.x, key), match4(v.y, key), match4(v.z, key), match4(v.w, key));
}
// bytes [a, b) of a 16-byte lane (a, b clamped to 0..16) as 16 bits
__device__ __forceinline__ uint32_t range16(int a, int b) {
  a = a < 0 ? 0 : (a > 16 ? 16 : a);
  b = b < 0 ? 0 : (b > 16 ? 16 : b);
  return b <= a ? 0u : ((0xFFFFu >> (16 - (b - a))) << a);
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
// this lane's bit of a wave-uniform 64-bit mask, as 1 - bit (one v_cndmask on the SGPR pair)
__device__ __forceinline__ uint32_t not_bit(uint64_t m) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, 1, 0, %1" : "=v"(r) : "s"(rfl64(m)));
  return r;
}
// 0 in lanes whose bit of m is set, -1 elsewhere
__device__ __forceinline__ uint32_t neg_notbit(uint64_t m) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, -1, 0, %1" : "=v"(r) : "s"(rfl64(m)));
  return r;
}
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

// Issue priority (s_setprio takes an immediate).  The 4 data waves sharing a SIMD otherwise get issue
// slots by age.  A data wave's priority is how far it trails the workgroup's front wave, so the waves a
// unit's AGG waits for take issue slots from the ones that run ahead (DataWave::step; a per-unit rotation
// measured -14 % on DELIM, no priorities -9 %).
__device__ __forceinline__ void set_prio(uint32_t p) {
  switch (p & 3u) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
  }
}

// the element type of an output form: 0 uint32, 1 uint64, 2 uint16 low words, 3 uint8 low bytes
template <int OUT64>
using OutOf = typename std::conditional<OUT64 == 1, uint64_t, typename std::conditional<OUT64 == 2, uint16_t,
              typename std::conditional<OUT64 == 3, uint8_t, uint32_t>::type>::type>::type;

template <typename T, bool NT = false>
__device__ __forceinline__ void put(void* out, uint64_t i, uint64_t v) {
  if constexpr (NT) __builtin_nontemporal_store((T)v, reinterpret_cast<T*>(out) + i);
  else reinterpret_cast<T*>(out)[i] = (T)v;
}

// Summary of a byte range as a function of the incoming line state S (does the current line already
// hold an emitted header?): count and outgoing state for S = false (F) and S = true (T).
struct Func {
  uint64_t cF, cT;
  uint32_t sF, sT;
};
__device__ __forceinline__ uint64_t pack_agg(const Func& f) {
  return kStatAgg | ((uint64_t)f.sT << 49) | ((uint64_t)f.sF << 48) | ((f.cT & 0xFFFFFFull) << 24) |
         (f.cF & 0xFFFFFFull);
}
__device__ __forceinline__ uint64_t pack_prefix(uint64_t count, uint32_t s) {
  return kStatPrefix | ((uint64_t)s << 48) | (count & 0xFFFFFFFFFFFFull);
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
  LB r;
  r.cF = sel64(bp, b.cF, a.cF + sel64(asF, b.cT, b.cF));
  r.cT = sel64(bp, b.cT, a.cT + sel64(asT, b.cT, b.cF));
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
constexpr int kWaveShl1 = 0x130;                          // lane l <- lane l + 1
constexpr int kWaveShr1 = 0x138;                          // lane l <- lane l - 1

template <int CTRL, int ROWS>
__device__ __forceinline__ LB lb_dpp(const LB& f) {       // identity where there is no source lane
  LB o;
  o.cF = dpp64<CTRL, ROWS>(f.cF, 0ull);
  o.cT = dpp64<CTRL, ROWS>(f.cT, 0ull);
  o.fl = dpp32<CTRL, ROWS>(f.fl, 2u);
  return o;
}

constexpr uint64_t kIdentDesc = kStatMask;   // status 3: "no unit here" (identity, always valid)

// Look-back window of unit u (lane 63 = nearest): slot k = desc[u-1-k] for k < W, slot W = the
// workgroup's own previous unit, whose inclusive prefix the coordinator substitutes when it reduces the
// window (it may not be known yet when the loads are issued), identity past it.  W = the number of units
// between the two (u itself for the workgroup's first unit, whose "previous unit" is the empty prefix).
// (With the static unit striding W = G - 1 < kLbSlots; a larger W would mean no base: the window then
// resolves only once it holds an inclusive prefix.)
constexpr int kLbPer = 4;                          // descriptors per lane (2: FASTA -22 %, 8: -9 to -16 %)
constexpr uint32_t kLbSlots = kLbPer * kWave;      // descriptors per window (256 >= G)
constexpr uint32_t kNoUnit = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t lb_span(uint32_t u, uint32_t u_prev) {
  const uint32_t d = u_prev == kNoUnit ? u : u - u_prev - 1u;
  return d < kLbSlots ? d : kLbSlots;
}
// All kLbPer loads are issued before any is used (a lane outside the window loads desc[0] and discards it):
// a load under its own branch got its own vmcnt(0) wait there, one round trip per slot.
__device__ __forceinline__ void lb_load(const ScanArgs& A, uint32_t u, uint32_t W, int lane, uint64_t (&d)[kLbPer]) {
  const uint32_t rl = (uint32_t)(kWave - 1 - lane);
#pragma unroll
  for (int j = 0; j < kLbPer; ++j) {
    const uint32_t k = kLbPer * rl + j;
    d[j] = ld_desc(&A.desc[k < W ? u - 1 - k : 0u]);
  }
#pragma unroll
  for (int j = 0; j < kLbPer; ++j) {
    const uint32_t k = kLbPer * rl + j;
    // an earlier launch's descriptor: not published yet
    d[j] = k < W ? ((d[j] & kEpochMask) == A.epoch ? d[j] : 0ull) : kIdentDesc;
  }
}

// Reduce one loaded window (one wave): prefix count P and line state S entering unit u, if every
// descriptor it needs is published (nearest first, down to the nearest inclusive prefix or the base).
// One parallel load + a DPP scan: no serial chain of prefixes.
__device__ __forceinline__ bool lb_reduce(uint64_t (&d)[kLbPer], uint32_t W, uint64_t basedesc, int lane,
                                          uint64_t& P, uint32_t& S_in) {
  const uint32_t rl = (uint32_t)(kWave - 1 - lane);
  uint32_t seen = 0, bad = 0;
#pragma unroll
  for (int j = 0; j < kLbPer; ++j) {                // nearest first
    if (kLbPer * rl + j == W) d[j] = basedesc;
    const uint64_t st = d[j] & kStatMask;
    if (!seen && st == 0ull) bad = 1;
    if (st == kStatPrefix) seen = 1;
  }
  const uint64_t PB = __ballot(seen);
  const uint64_t BB = __ballot(bad);
  if (PB == 0ull) return false;                     // no base and no inclusive prefix in the window yet
  // lanes from the nearest one (63) down to the nearest lane holding a prefix must all be published
  const uint64_t need = PB ? ~((1ull << (63 - __builtin_clzll(PB))) - 1ull) : ~0ull;
  if (BB & need) return false;
  // Fast path.  Line-state maps of units are constant (the unit holds a '\n') or the identity (it does
  // not); with only constant maps between the nearest prefix and u, every unit's incoming state is the
  // state bit (bit 48 of AGG and PREFIX descriptors alike) of its farther neighbour, so the prefix is a
  // plain sum of selected counts.  Any identity map in range: the full functional scan below.
  {
    const int Lp = 63 - __builtin_clzll(PB);          // nearest lane holding a prefix (PB != 0)
    uint32_t jp = kLbPer;
#pragma unroll
    for (int j = kLbPer - 1; j >= 0; --j)
      if ((d[j] & kStatMask) == kStatPrefix) jp = (uint32_t)j;
    const uint32_t kP = (uint32_t)kLbPer * (uint32_t)(63 - Lp) + (uint32_t)__builtin_amdgcn_readlane((int)jp, Lp);
    // state out of each slot and of the farther neighbour of the lane's last slot (lane - 1's slot 0)
    uint32_t so[kLbPer];
#pragma unroll
    for (int j = 0; j < kLbPer; ++j) so[j] = (uint32_t)(d[j] >> 48) & 1u;
    const uint32_t so_far = dpp32<kWaveShr1, 0xF>(so[0], 0u);
    uint32_t sum = 0, ident = 0;
#pragma unroll
    for (int j = 0; j < kLbPer; ++j) {
      const uint32_t k = kLbPer * rl + j;
      if (k < kP) {
        const uint32_t sin = j < kLbPer - 1 ? so[j + 1] : so_far;
        const uint32_t cF = (uint32_t)d[j] & 0xFFFFFFu, cT = (uint32_t)(d[j] >> 24) & 0xFFFFFFu;
        sum += sin ? cT : cF;
        ident |= (uint32_t)((d[j] >> 48) ^ (d[j] >> 49)) & 1u;
      }
    }
    if (__ballot(ident) == 0ull) {
      uint64_t pv = 0;
#pragma unroll
      for (int j = 0; j < kLbPer; ++j)
        if ((uint32_t)j == jp) pv = d[j] & 0xFFFFFFFFFFFFull;
      // wave sum of the selected counts (< 2^32: at most 511 units of < 2^17 events)
      sum += dpp32<kRowShr1, 0xF>(sum, 0u);
      sum += dpp32<kRowShr2, 0xF>(sum, 0u);
      sum += dpp32<kRowShr4, 0xF>(sum, 0u);
      sum += dpp32<kRowShr8, 0xF>(sum, 0u);
      sum += dpp32<kRowBcast15, 0xA>(sum, 0u);
      sum += dpp32<kRowBcast31, 0xC>(sum, 0u);
      P = readlane64(pv, Lp) + (uint32_t)__builtin_amdgcn_readlane((int)sum, kWave - 1);
      S_in = (uint32_t)__builtin_amdgcn_readlane((int)so[0], kWave - 1);
      return true;
    }
  }
  LB f = lb_from_desc(d[kLbPer - 1]);
#pragma unroll
  for (int j = kLbPer - 2; j >= 0; --j) f = lb_then(f, lb_from_desc(d[j]));
  // inclusive scan, lane 0 (farthest) -> lane 63 (nearest): farther composed in front of nearer
  f = lb_then(lb_dpp<kRowShr1, 0xF>(f), f);
  f = lb_then(lb_dpp<kRowShr2, 0xF>(f), f);
  f = lb_then(lb_dpp<kRowShr4, 0xF>(f), f);
  f = lb_then(lb_dpp<kRowShr8, 0xF>(f), f);
  f = lb_then(lb_dpp<kRowBcast15, 0xA>(f), f);
  f = lb_then(lb_dpp<kRowBcast31, 0xC>(f), f);
  P = readlane64(f.cF, kWave - 1);
  S_in = (uint32_t)__builtin_amdgcn_readlane((int)f.fl, kWave - 1) & 1u;
  return true;
}

// ------------------------------------------------------------------------------------------ geometry
// Unit -> chunk lookup over the chunk table (read-only, read through the constant address space so it
// compiles to scalar loads and never enters the vector-memory counter the data waves' hand-waited loads
// rely on).  A cursor follows the increasing units of one wave, falling back to a binary search when it
// would skip chunks.
typedef __attribute__((address_space(4))) const uint64_t cu64;   // constant address space: s_load
struct Tab {
  cu64* lo;
  cu64* hi;
  cu64* u0;                          // [nchunks + 1]
};
struct Cursor {
  uint64_t lo, hi;                   // chunk c = [lo, hi) covers units [u0, u1)
  uint32_t c, u0, u1, valid;
};
struct Geo {                          // one unit (wave-uniform); lo_u / hi_u relative to ubase
  uint64_t ubase;
  uint32_t lo_u, hi_u, c, fl;         // fl: bit0 first unit of its chunk, bit1 last, bit2 valid
};
constexpr uint32_t kGeoFirst = 1u, kGeoLast = 2u, kGeoValid = 4u;
__device__ __forceinline__ Geo geo_of(const Tab& T, uint32_t nchunks, uint32_t nunits, uint32_t u, Cursor& cur) {
  Geo g;
  if (u >= nunits) {
    g.ubase = 0;
    g.lo_u = g.hi_u = g.c = g.fl = 0;
    return g;
  }
  if (!cur.valid || u < cur.u0 || u >= cur.u1) {
    uint32_t c = 0, cn = nchunks;
    if (cur.valid && u >= cur.u1 && cur.c + 1 < nchunks && (uint32_t)T.u0[cur.c + 2] > u) {
      c = cur.c + 1;                                   // common case: the next chunk
    } else {
      while (cn - c > 1) {
        const uint32_t m = (c + cn) >> 1;
        if ((uint32_t)T.u0[m] <= u) c = m; else cn = m;
      }
    }
    cur.c = c;
    cur.u0 = (uint32_t)T.u0[c];
    cur.u1 = (uint32_t)T.u0[c + 1];
    cur.lo = T.lo[c];
    cur.hi = T.hi[c];
    cur.valid = 1;
  }
  g.c = cur.c;
  g.ubase = (cur.lo & ~15ull) + (uint64_t)(u - cur.u0) * (uint64_t)kUnitBytes;
  g.lo_u = cur.lo > g.ubase ? (uint32_t)(cur.lo - g.ubase) : 0u;      // 0..15, first unit only
  const uint64_t hu = cur.hi - g.ubase;                                // > 0: a unit holds chunk bytes
  g.hi_u = hu < (uint64_t)(kUnitBytes + 64) ? (uint32_t)hu : (uint32_t)(kUnitBytes + 64);
  g.fl = kGeoValid | (u == cur.u0 ? kGeoFirst : 0u) | (u + 1 == cur.u1 ? kGeoLast : 0u);
  return g;
}
// the chunk bounds [lo_w, hi_w) relative to data wave w's 8 KiB range of unit g
__device__ __forceinline__ int wave_lo(const Geo& g, int wave) {
  const int v = (int)g.lo_u - wave * kWaveBytes;
  return v > 0 ? v : 0;
}
__device__ __forceinline__ int wave_hi(const Geo& g, int wave) {
  const int v = (int)g.hi_u - wave * kWaveBytes;
  return v < 0 ? 0 : (v > kWaveBytes + 16 ? kWaveBytes + 16 : v);
}

// ------------------------------------------------------------------------------------------ input loads
typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

struct Buf {
  v4u x[kRows];              // raw load destinations (owned by the in-flight asm loads until wait_buf)
  uint32_t la;               // first dword after this buffer (next-byte lookahead of its last row)
};

// Unconditional bounds-checked loads of one buffer (kRows KiB + lookahead): bytes at or past the 16-byte
// block holding the chunk end read as 0 (num_records), so every wave always has exactly kLoadsPerBuf
// loads in flight per buffer.  Issued as inline asm: the compiler inserts no wait for them, and the
// data waves wait with ONE explicit `s_waitcnt vmcnt((kBufs - 1) * kLoadsPerBuf)` per buffer: a wave
// scans one buffer while its kBufs - 1 others are in flight.  Phase-B stores are issued before the last
// prefetch of a step, so at each wait the youngest vector-memory operations are the other buffers' loads
// (plus, at the first wait of a step, those stores: a slightly conservative wait).  tools/isa_guard.py
// checks the compiled code never touches a destination while its load can still be in flight.
constexpr int kLoadsPerBuf = kRows + 1;
// Input bytes are read once: non-temporal loads (nt) stream them without displacing L2 lines; measured on
// MI355X the load pattern alone goes from 6.2 to 6.9 TB/s (a load-only probe, round 1).
#define DP_LDPOL "nt"

// buffer resource for one wave range: num_records ends at the 16-byte block holding the chunk end
__device__ __forceinline__ v4i buf_rsrc(const uint8_t* base, uint64_t wbase, int hi_w) {
  const uint32_t nrec = (uint32_t)((hi_w + 15) & ~15);
  const uint64_t addr = (uint64_t)(uintptr_t)(base + wbase);
  v4i r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)addr);
  r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(addr >> 32) & 0xFFFF);   // stride 0
  r[2] = __builtin_amdgcn_readfirstlane((int)nrec);
  r[3] = 0x00020000;
  return r;
}

// rows 0..R-1 of a buffer: 12-bit immediate offsets, so a second VGPR offset from row 4 on
template <int R>
__device__ __forceinline__ void load_rows(Buf& b, uint32_t off0, const v4i& r) {
  if constexpr (R > 0) {
    load_rows<R - 1>(b, off0, r);
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3 " DP_LDPOL
                 : "=v"(b.x[R - 1]) : "v"(off0 + (uint32_t)((R - 1) >> 2) * 4096u), "s"(r), "i"(((R - 1) & 3) * kRowBytes)
                 : "memory");
  }
}
// buffer h of data wave w's range of unit g (bytes [h*kBufBytes, (h+1)*kBufBytes + 4))
__device__ __forceinline__ void load_buf(Buf& b, const ScanArgs& A, const Geo& g, int wave, int lane, int half) {
  int hb = (g.fl & kGeoValid) ? wave_hi(g, wave) - half * kBufBytes : 0;
  hb = hb < 0 ? 0 : (hb > kBufBytes + 16 ? kBufBytes + 16 : hb);
  const v4i r = buf_rsrc(A.base, g.ubase + (uint64_t)wave * kWaveBytes + (uint64_t)half * kBufBytes, hb);
  static_assert(kRowBytes == 1024, "load_rows offsets assume rows of 1 KiB");
  load_rows<kRows>(b, (uint32_t)lane * 16u, r);
  asm volatile("buffer_load_dword %0, %1, %2, 0 offen " DP_LDPOL : "=v"(b.la) : "v"((uint32_t)kBufBytes), "s"(r) : "memory");
}

// Wait for this buffer's loads, then "redefine" every destination register: the empty asm makes each
// value live until here (an unused destination must not be reallocated while its load is in flight)
// and nothing that reads the data can be scheduled above the wait.  The (kBufs - 1) * kLoadsPerBuf
// youngest vector-memory operations are the other buffers' loads, still in flight.
__device__ __forceinline__ void touch_buf(Buf& b) {
#pragma unroll
  for (int r = 0; r < kRows; ++r) asm volatile("" : "+v"(b.x[r]) :: "memory");
  asm volatile("" : "+v"(b.la) :: "memory");
}
__device__ __forceinline__ void wait_buf(Buf& b) {
  asm volatile("s_waitcnt vmcnt(%0)" :: "i"((kBufs - 1) * kLoadsPerBuf) : "memory");
  touch_buf(b);
  __builtin_amdgcn_sched_barrier(0);
}
// After the last step every buffer still has (unused) loads in flight: wait for them and keep their
// destinations live until then, or the compiler reuses those VGPRs and the landing loads clobber them.
__device__ __forceinline__ void drain_bufs(Buf (&b)[kBufs]) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int h = 0; h < kBufs; ++h) touch_buf(b[h]);
  __builtin_amdgcn_sched_barrier(0);
}

// The same buffers without the lookahead dword (a FASTA row needs the byte after it; a delimiter row does not):
// kRows loads per buffer, 2 VGPRs fewer per wave (line_kernel runs at the 128-VGPR limit).  The two-kernel and
// lockstep kernels use these; FASTA reads its lookahead dword by a scalar load (lookahead_s).
struct BufN {
  v4u x[kRows];
};
constexpr int kLoadsPerBufN = kRows;
__device__ __forceinline__ void load_bufx(BufN& b, const ScanArgs& A, const Geo& g, int lane, int half) {
  int hb = (g.fl & kGeoValid) ? wave_hi(g, 0) - half * kBufBytes : 0;
  hb = hb < 0 ? 0 : (hb > kBufBytes + 16 ? kBufBytes + 16 : hb);
  const v4i r = buf_rsrc(A.base, g.ubase + (uint64_t)half * kBufBytes, hb);
  Buf& bb = *reinterpret_cast<Buf*>(&b);          // (load_rows writes x[] only)
  load_rows<kRows>(bb, (uint32_t)lane * 16u, r);
}
__device__ __forceinline__ void touch_bufx(BufN& b) {
#pragma unroll
  for (int r = 0; r < kRows; ++r) asm volatile("" : "+v"(b.x[r]) :: "memory");
}
__device__ __forceinline__ void wait_bufx(BufN& b) {
  asm volatile("s_waitcnt vmcnt(%0)" :: "i"((kBufs - 1) * kLoadsPerBufN) : "memory");
  touch_bufx(b);
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void drain_bufsx(BufN (&b)[kBufs]) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int h = 0; h < kBufs; ++h) touch_bufx(b[h]);
  __builtin_amdgcn_sched_barrier(0);
}
typedef __attribute__((address_space(4))) const uint32_t cu32s;   // constant address space: s_load_dword
// the first dword after buffer h of a wave range (FASTA's next-byte lookahead) by a scalar load through the
// constant address space (it waits on lgkmcnt, never on the hand-counted vmcnt); read only where that byte lies
// inside the chunk, the range's own first dword elsewhere (always in the buffer).  (As a ninth vector load per
// buffer it measured 669-672 vs 676-678 us per 4 GiB, profiles/r04/ab/map_bufn.)
__device__ __forceinline__ uint32_t lookahead_s(const uint8_t* base, const Geo& g, int h, bool interior, int hi) {
  const bool inb = interior || (h + 1) * kBufBytes < hi;
  const uint64_t at = g.ubase + (inb ? (uint64_t)(h + 1) * kBufBytes : 0ull);
  return *(cu32s*)(uintptr_t)(base + at);
}

// ------------------------------------------------------------------------------------------ LDS state
struct WaveRec {                   // one data wave's phase-A result for one unit (written by its lane 0)
  uint64_t wbase;                  // aligned coordinate of the wave range's first byte
  uint32_t lohi;                   // the chunk bounds in the range: lo_w | hi_w << 16 (dense rescan)
  uint32_t cF, cT;                 // count if the range is entered with state false / true
  uint32_t fl;                     // bit0 sF, bit1 sT (state after the range), bit2 fV, bit3 dense
  uint32_t fn;                     // FASTA: 1 + offset of the range's first '\n', 0 if none
  uint32_t ev0, nev;               // the range's events in the wave's circular list (running index, count)
};
constexpr uint32_t kFlDense = 8u;

struct Shared {
  uint16_t ev[kDataWaves][kEvCap];                          // per-wave circular event lists
  WaveRec rec[kRing][kDataWaves];
  uint32_t exF[kRing][kDataWaves], exT[kRing][kDataWaves];  // per-wave exclusive prefix functions
  uint32_t es[kRing][kDataWaves];                           // bit0 esF, bit1 esT
  uint32_t uF[kRing], uT[kRing], us[kRing];                 // the unit's function (us: bit0 sF, bit1 sT)
  uint64_t P[kRing][kDataWaves];                            // per-wave true prefix (coordinator)
  uint32_t S[kRing][kDataWaves];                            // per-wave true incoming line state
  uint32_t done[kRing];                                     // data waves finished phase A of the slot's unit
  uint32_t ready[kRing];                                    // = unit index + 1 once P/S of the slot are set
  uint32_t front;                                           // highest step a data wave of the workgroup has started
  uint32_t uq[kUnitQ];                                      // unit claimed for step k at [k % kUnitQ] (coordinator)
  uint32_t uq_ready[kUnitQ];                                // = k + 1 once uq of step k is set
};

// ------------------------------------------------------------------------------------------ rows
// Events of one row: per-lane mask em (bit i = byte i of the lane), ranks from rank0 in byte order.
// store(rank, byte offset in the lane) per event; returns the wave's event count in the row.
template <class Store>
__device__ __forceinline__ uint32_t emit_row(uint32_t em, uint32_t rank0, Store&& store) {
  const uint32_t c = (uint32_t)__popc(em);
  const uint64_t any1 = __ballot(c != 0u);
  if (__ballot(c > 1u) == 0ull) {                    // common: at most one event per lane, no loop
    if (em) store(rank0 + mbcnt(any1), (uint32_t)__builtin_ctz(em));
    return (uint32_t)__popcll(any1);
  }
  uint32_t tot;
  const uint32_t ex = wave_excl<5>(c, tot);
  uint32_t rk = rank0 + ex;
  for (uint32_t x = em; x; x &= x - 1u, ++rk) store(rk, (uint32_t)__builtin_ctz(x));
  return tot;
}

struct FState {                    // wave-uniform FASTA scan state over one wave range
  uint32_t S;                      // the current line already holds an emitted header
  uint32_t nlseen;                 // a '\n' was seen in the range
  uint32_t fV;                     // state just before the range's first '\n'
  int fn;                          // offset of the range's first '\n' in the range, -1 if none
  uint32_t cnt;                    // emitted headers
  uint32_t nev;                    // events (starts and ends)
};

// FASTA rows of one wave range ([wbase, wbase + 8 KiB) in aligned coordinates, chunk [lo, hi)).
// fasta.py:36 emits at p iff d[p] == '>', no header was emitted earlier on p's line inside the chunk,
// p + 1 < c1 and d[p + 1] != '\n'; its end is the next '\n' + 1.  Per lane, 16-bit masks
// NL / GT; V = valid '>' bits.  "First valid '>' of every line segment" is one carry trick:
// R = ~(V | NL) + (NL << 1) + [segment start at the lane start]: carries run through bytes that are
// neither, so R has a 1 exactly where the carry from each line start stops.  The line state at each lane
// start is a 64-bit carry chain over two ballots (generate: a valid '>' after the lane's last '\n';
// propagate: no '\n' in the lane), on the scalar unit.  Rows entered with S = false and without any '>'
// are skipped after one exact test.
// One row r (row0 = r KiB into the range): xr = the lane's 16 bytes, wn = a word whose lane-0 byte 0 is the
// byte after the row (only read when that byte is inside the chunk).
// INTERIOR: the whole range and the byte after it lie inside the chunk (no edge rows; every row's next
// byte is valid): the same code without the per-row edge tests.
template <bool INTERIOR, class Store>
__device__ __forceinline__ void fasta_row(const v4u& xr, uint32_t wn, int r, int lo, int hi, int lane, FState& st,
                                          Store&& store) {
  {
    const int row0 = r * kRowBytes;
    const bool edge = !INTERIOR && (row0 < lo || row0 + kRowBytes >= hi);
    const uint32_t g0 = match4(xr[0], kKeyGT), g1 = match4(xr[1], kKeyGT);
    const uint32_t g2 = match4(xr[2], kKeyGT), g3 = match4(xr[3], kKeyGT);
    const bool anygt = __ballot((g0 & g1 & g2 & g3) != 0xFFFFFFFFu) != 0ull;
    if (!edge && !st.S && st.nlseen && !anygt) return;
    uint32_t NL = pack16(match4(xr[0], kKeyNL), match4(xr[1], kKeyNL), match4(xr[2], kKeyNL), match4(xr[3], kKeyNL));
    uint32_t GT = anygt ? pack16(g0, g1, g2, g3) : 0u;
    uint32_t nxt63 = 0, lastm = 0;
    if (INTERIOR || row0 + kRowBytes < hi) nxt63 = ((uint32_t)__builtin_amdgcn_readlane((int)wn, 0) & 0xFFu) == 10u;
    if (edge) {
      const int rel_lo = lo - row0 - 16 * lane;
      const int rel_hi = hi - row0 - 16 * lane;
      const uint32_t rm = range16(rel_lo, rel_hi);
      NL &= rm;
      GT &= rm;
      if (rel_hi >= 1 && rel_hi <= 16) lastm = 1u << (rel_hi - 1);   // p + 1 < c1
    }
    // next byte is '\n': this lane's bits shifted down, the next lane's bit 0 on top (lane 63: the byte
    // after the row); bits above 15 of the shifted-in word do not matter (GT is 16 bits)
    const uint32_t dn = dpp32<kWaveShl1, 0xF>(NL, nxt63);
    const uint32_t V = GT & ~((NL >> 1) | (dn << 15) | lastm);
    const uint64_t H = __ballot(NL != 0u);
    const uint32_t m1 = neg_notbit(H);                            // -1: no '\n' in the lane (lane start = segment start)
    const uint32_t R1 = (((V | NL) ^ 0xFFFFu) + (NL << 1)) - m1;
    const uint64_t SB = __ballot(R1 < 0x10000u);                  // a valid '>' after the lane's last '\n'
    // start(p + 1) = SB(p) | (~H(p) & start(p)), start(0) = S: the carries of a + SB + S with a = SB | ~H
    const uint64_t a = SB | ~H;
    const uint64_t Sst = (a + SB + (uint64_t)st.S) ^ a ^ SB;     // line state at each lane start
    // the lane start opens a segment only if its state is false: add it there, take it back elsewhere
    const uint32_t R = R1 + not_bit(Sst) + m1;
    const uint32_t emits = V & R;
    const uint32_t em = emits | (NL & ~R);
    if (!st.nlseen && H) {
      const int j0 = (int)__builtin_ctzll(H);
      const uint32_t low = NL & (0u - NL);
      const uint32_t vb = (V & (low - 1u)) != 0u;
      st.fV = (uint32_t)((Sst >> j0) & 1ull) | (uint32_t)__builtin_amdgcn_readlane((int)vb, j0);
      st.fn = r * kRowBytes + j0 * 16 + __builtin_ctz((uint32_t)__builtin_amdgcn_readlane((int)NL, j0));
      st.nlseen = 1;
    }
    if (__ballot(em != 0u)) {
      const uint32_t pos0 = (uint32_t)(r * kRowBytes + lane * 16);
      const uint32_t tot = emit_row(em, st.nev, [&](uint32_t rk, uint32_t b) { store(rk, pos0 + b); });
      st.cnt += (tot + (st.S ^ 1u)) >> 1;                         // events alternate start, end, ...
      st.nev += tot;
    }
    st.S = (uint32_t)((SB | (~H & Sst)) >> 63);                 // the state after lane 63
  }
}
// one buffer: rows half*8 .. half*8 + 7 of the wave range
template <bool INTERIOR, class Store>
__device__ __forceinline__ void fasta_rows(const v4u (&x)[kRows], uint32_t la, int half, int lo, int hi, int lane,
                                           FState& st, Store&& store) {
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    const int R = half * kRows + r;
    if (!INTERIOR && R * kRowBytes >= hi) break;
    fasta_row<INTERIOR>(x[r], (r + 1 < kRows) ? x[(r + 1) & (kRows - 1)][0] : la, R, lo, hi, lane, st, store);
  }
}

// Delimiter rows of one wave range: events = delimiter bytes.  nev counts them.
template <bool INTERIOR, class Store>
__device__ __forceinline__ void delim_row(const v4u& xr, int r, int lo, int hi, uint32_t key, int lane, uint32_t& nev,
                                          Store&& store) {
  const int row0 = r * kRowBytes;
  const bool edge = !INTERIOR && (row0 < lo || row0 + kRowBytes >= hi);
  const uint32_t p0 = match4(xr[0], key), p1 = match4(xr[1], key);
  const uint32_t p2 = match4(xr[2], key), p3 = match4(xr[3], key);
  if (!edge && __ballot((p0 & p1 & p2 & p3) != 0xFFFFFFFFu) == 0ull) return;
  uint32_t M = pack16(p0, p1, p2, p3);
  if (edge) M &= range16(lo - row0 - 16 * lane, hi - row0 - 16 * lane);
  if (__ballot(M != 0u)) {
    const uint32_t pos0 = (uint32_t)(row0 + lane * 16);
    nev += emit_row(M, nev, [&](uint32_t rk, uint32_t b) { store(rk, pos0 + b); });
  }
}
template <bool INTERIOR, class Store>
__device__ __forceinline__ void delim_rows(const v4u (&x)[kRows], int half, int lo, int hi, uint32_t key, int lane,
                                           uint32_t& nev, Store&& store) {
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    const int R = half * kRows + r;
    if (!INTERIOR && R * kRowBytes >= hi) break;
    delim_row<INTERIOR>(x[r], R, lo, hi, key, lane, nev, store);
  }
}

// ------------------------------------------------------------------------------------------ phase A / B
// Phase A of one unit on one data wave, one buffer (half) at a time: events to the wave's list (ranks
// from ev_head), then the range's summary to rec.
struct PhaseA {
  FState st;                       // FASTA state; DELIM uses st.nev only
  uint64_t wbase;
  int lo, hi;
};
template <int MODE, int OUT64>
__device__ __forceinline__ void phase_a_half(const ScanArgs& A, PhaseA& pa, Buf& b, int half, int wave, int lane,
                                             Shared& sh, uint32_t ev_head) {
  v4u x[kRows];
#pragma unroll
  for (int r = 0; r < kRows; ++r) x[r] = b.x[r];
  uint16_t* evw = sh.ev[wave];
  // Ranks past kDenseMax (a dense range: its list is never read) all land on the range's last reserved
  // entry, which the room check keeps free: a clamp instead of a conditional store.
  auto keep = [&](uint32_t rk, uint32_t pos) {
    evw[(ev_head + (rk < kDenseMax - 1u ? rk : kDenseMax - 1u)) & kEvMask] = (uint16_t)pos;
  };
  const bool interior = pa.lo == 0 && pa.hi > kWaveBytes;   // wave-uniform
  (void)interior;
  if constexpr (MODE == kFasta) {
    if (interior) fasta_rows<true>(x, b.la, half, pa.lo, pa.hi, lane, pa.st, keep);
    else fasta_rows<false>(x, b.la, half, pa.lo, pa.hi, lane, pa.st, keep);
  } else {
    // DELIM: no specialized copy (measured ±1% with uint64 output; with uint32 output the copy pushes
    // the kernel past 128 VGPRs and spills an in-flight load destination, which tools/isa_guard.py flags)
    delim_rows<false>(x, half, pa.lo, pa.hi, A.delim ^ kSel12, lane, pa.st.nev, keep);
  }
}
template <int MODE>
__device__ __forceinline__ void phase_a_rec(PhaseA& pa, const Geo& g, int wave, uint32_t ev_head, WaveRec& rec) {
  FState& st = pa.st;
  uint32_t fl;
  if constexpr (MODE == kFasta) {
    if (!st.nlseen) st.fV = st.S;
    uint32_t cT = st.cnt - st.fV, sT = st.nlseen ? st.S : 1u;
    if ((g.fl & kGeoFirst) && wave == 0) { cT = st.cnt; sT = st.S; }   // chunk start: the state is reset
    rec.cF = st.cnt;
    rec.cT = cT;
    fl = st.S | (sT << 1) | (st.fV << 2);
    rec.fn = (uint32_t)(st.fn + 1);
  } else {
    rec.cF = rec.cT = st.nev;
    fl = 0;
    rec.fn = 0;
  }
  const bool dense = st.nev > kDenseMax;
  rec.wbase = pa.wbase;
  rec.lohi = (uint32_t)pa.lo | ((uint32_t)pa.hi << 16);
  rec.fl = fl | (dense ? kFlDense : 0u);
  rec.ev0 = ev_head;
  rec.nev = dense ? 0u : st.nev;
}

// uint8 output (out_mode 4): the low 16 bits of `count`, the entries before the 256-byte boundary at range position
// `key` (16-byte aligned, as every range starts 16-byte aligned and object offsets are congruent to device addresses
// mod 16), when that boundary is one of the launch's and lies inside the range's chunk bytes [lo, hi): each boundary
// of the contiguous ranges is then written by exactly one range.  Within a 64 KiB block the counts before its 256
// boundaries differ from the block table's entry by at most 255 x 256 < 2^16, so 16 bits locate every entry.
__device__ __forceinline__ void put_sub(const ScanArgs& A, uint64_t off0, int key, int lo, int hi, uint64_t count) {
  const uint64_t b = off0 + (uint64_t)key;
  if ((b & 255u) != 0u || key < lo || key >= hi || key >= kWaveBytes) return;
  const uint64_t s = (b >> 8) - A.sub_s0;
  if ((b >> 8) >= A.sub_s0 && s < A.sub_n) __builtin_nontemporal_store((uint16_t)count, A.subtab + s);
}
// ... for a range's sorted position list: lane l takes the range's l-th 256-byte boundary (a range of 16 KiB holds
// exactly 64) and counts the positions before it by a binary search over the list.  (Counting the boundaries between
// consecutive entries instead, through an LDS scratch run, measured 7 % slower on CSV and 3 % on VCF.)
template <class Ev>
__device__ __forceinline__ void place_subs(const ScanArgs& A, Ev&& ev, uint32_t nev, uint64_t P, uint64_t off0, int lo,
                                           int hi, int lane) {
  const int key = (int)(((off0 + 255u) & ~255ull) - off0) + 256 * lane;
  uint32_t a = 0, b = nev;
  while (a < b) {
    const uint32_t m = (a + b) >> 1;
    if ((int)ev(m) < key) a = m + 1u;
    else b = m;
  }
  put_sub(A, off0, key, lo, hi, P + a);
}

// Dense phase B: rescan the range from the input with its true state and count, writing the output
// directly.  Plain loads (the compiler waits for them; the older in-flight prefetch only makes those
// waits conservative).  Runs only where the other buffer's registers are free (after phase A).
template <int MODE, int OUT64>
__device__ __forceinline__ void dense_b(const ScanArgs& A, uint64_t wbase, uint32_t lohi, uint64_t P, uint32_t S,
                                        int lane) {
  typedef OutOf<OUT64> OutT;
  const int lo = (int)(lohi & 0xFFFFu), hi = (int)(lohi >> 16);
  const int hi16 = (hi + 15) & ~15;
  const uint8_t* src = A.base + wbase;
  auto row_in = [&](int r) {
    const int a = r * kRowBytes + lane * 16;
    return a + 16 <= hi16 ? *reinterpret_cast<const v4u*>(src + a) : v4u{0u, 0u, 0u, 0u};
  };
  const uint64_t obj_off = A.obj_base - A.shift + wbase;
  const bool near4g = OUT64 == 0 && !A.wrap32 && obj_off + kWaveBytes + 1 > 0xFFFFFFFFull;
  bool ovf = false;
  if constexpr (MODE == kFasta) {
    const uint64_t b0 = 2 * P - S, last = 2 * A.cap - 1;
    FState st{S, 1u, 0u, -1, 0u, 0u};
    auto out = [&](uint32_t rk, uint32_t pos) {
      const uint64_t slot = b0 + rk;
      const uint64_t val = obj_off + pos + (slot & 1u);
      if (near4g) ovf |= val > 0xFFFFFFFFull;
      put<OutT>(A.out, slot < last ? slot : last, val);
    };
#pragma unroll 1
    for (int r = 0; r < kRangeRows && r * kRowBytes < hi; ++r) {
      const int an = (r + 1) * kRowBytes;
      const uint32_t wn = an + 4 <= hi16 ? *reinterpret_cast<const uint32_t*>(src + an) : 0u;
      fasta_row<false>(row_in(r), wn, r, lo, hi, lane, st, out);
    }
  } else {
    const uint64_t last = A.cap - 1, add = obj_off + A.emit_add;
    const uint32_t k = A.every_k;
    // every k-th delimiter overall (counting from the carried ordinal): rank rk is kept iff rk >= r0 and
    // (rk - r0) % k == 0, at q0 + (rk - r0) / k
    const uint64_t Pc = P + A.carry;
    const uint32_t r0 = k == 1u ? 0u : (uint32_t)((k - 1u) - Pc % k);
    const uint64_t q0 = (Pc + r0) / k - A.carry / k;
    uint32_t n = 0;
    auto out = [&](uint32_t rk, uint32_t pos) {
      if (rk < r0) return;
      const uint32_t d = rk - r0;
      const uint32_t t = k == 1u ? d : d / k;
      if (t * k != d) return;
      const uint64_t q = q0 + t;
      const uint64_t val = add + pos;
      if (near4g) ovf |= val > 0xFFFFFFFFull;
      put<OutT, true>(A.out, q < last ? q : last, val);
    };
    const uint32_t key = A.delim ^ kSel12;
#pragma unroll 1
    for (int r = 0; r < kRangeRows && r * kRowBytes < hi; ++r) {
      const v4u x = row_in(r);
      if constexpr (OUT64 == 3) {
        // the 256-byte boundaries of this row: the lane whose 16 bytes start at one counts the delimiters before it
        const int a = r * kRowBytes + lane * 16;
        uint32_t tot;
        const uint32_t m = pack16(match4(x[0], key), match4(x[1], key), match4(x[2], key), match4(x[3], key));
        const uint32_t ex = wave_excl<5>((uint32_t)__popc(m & range16(lo - a, hi - a)), tot);
        put_sub(A, obj_off, a, lo, hi, P + n + ex);
      }
      delim_row<false>(x, r, lo, hi, key, lane, n, out);
    }
  }
  if (ovf) atomicOr(A.err, kErrOverflow);
}

// The stores of one range's delimiter list (a data wave's phase B, or the lockstep kernel's placement): list
// entry i is ev(i), a position relative to the range's first byte (object offset obj_off); the range's first
// delimiter has launch ordinal P.  every_k / emit_add / carry select and shift the entries (FASTQ read ends);
// stores go to min(q, cap - 1) (an overflowing launch reports DP_ERR_CAPACITY and is discarded).  Returns
// whether a uint32 value overflowed.
template <int OUT64, bool PAIR = true, class Ev>
__device__ __forceinline__ bool place_delims(const ScanArgs& A, Ev&& ev, uint32_t nev, uint64_t P, uint64_t obj_off,
                                             int lane) {
  typedef OutOf<OUT64> OutT;
  const bool near4g = OUT64 == 0 && !A.wrap32 && obj_off + kWaveBytes + 1 > 0xFFFFFFFFull;
  bool ovf = false;
  const uint64_t last = A.cap - 1, add = obj_off + A.emit_add;
  const uint32_t k = A.every_k;
  // every k-th delimiter overall (FASTQ read ends), counting from the carried ordinal: list entries
  // r0, r0 + k, ... go to q0, q0 + 1, ...  (k == 1, the newline index: no 64-bit divisions)
  uint32_t r0 = 0, nq = nev;
  uint64_t q0 = P;
  if (k != 1u) {
    const uint64_t Pc = P + A.carry;
    r0 = (uint32_t)((k - 1u) - Pc % k);
    q0 = (Pc + r0) / k - A.carry / k;
    nq = nev > r0 ? (nev - r0 + k - 1u) / k : 0u;
  }
  if constexpr (OUT64 == 1 && PAIR) {
    // Every delimiter, uint64 output, the whole list in bounds (wave-uniform): two offsets per lane and
    // one 16-byte store, which halves the store instructions that queue behind the input loads.  An odd
    // q0 puts its first entry in a single store so that the pairs are 16-byte aligned.
    if (k == 1u && q0 + nq <= A.cap && ((uintptr_t)A.out & 15u) == 0) {
      uint64_t* o = reinterpret_cast<uint64_t*>(A.out) + q0;
      const uint32_t h = nq ? (uint32_t)(q0 & 1u) : 0u;
      if (h && lane == 0) o[0] = add + ev(0u);
      const uint32_t m = nq - h;
      for (uint32_t t = 2u * (uint32_t)lane; t < m; t += 2u * kWave) {
        const uint32_t i = h + t;
        const uint64_t v0 = add + ev(i);
        if (t + 1u < m) {
          const uint64_t v1 = add + ev(i + 1u);
          __builtin_nontemporal_store(v2u64{v0, v1}, reinterpret_cast<v2u64*>(o + i));
        } else {
          __builtin_nontemporal_store((uint64_t)v0, o + i);
        }
      }
      return false;
    }
  }
  if constexpr (OUT64 == 2) {
    // uint16 low words, every delimiter, whole list in bounds: eight entries per lane, one 16-byte store;
    // the first (8 - q0 % 8) % 8 entries go alone so that the groups are 16-byte aligned
    if (k == 1u && q0 + nq <= A.cap && ((uintptr_t)A.out & 15u) == 0) {
      uint16_t* o = reinterpret_cast<uint16_t*>(A.out) + q0;
      const uint32_t hh = (uint32_t)((8u - (uint32_t)(q0 & 7u)) & 7u);
      const uint32_t h = hh < nq ? hh : nq;
      if ((uint32_t)lane < h) o[lane] = (uint16_t)(add + ev((uint32_t)lane));
      const uint32_t m = nq - h, g = m >> 3;
      for (uint32_t t = (uint32_t)lane; t < g; t += kWave) {
        const uint32_t i = h + 8u * t;
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t a = (uint32_t)(uint16_t)(add + ev(i + 2u * e));
          const uint32_t b = (uint32_t)(uint16_t)(add + ev(i + 2u * e + 1u));
          w[e] = a | (b << 16);
        }
        const v4u pk = {w[0], w[1], w[2], w[3]};
        __builtin_nontemporal_store(pk, reinterpret_cast<v4u*>(o + i));
      }
      for (uint32_t t = h + 8u * g + (uint32_t)lane; t < nq; t += kWave) o[t] = (uint16_t)(add + ev(t));
      return false;
    }
  }
  if constexpr (OUT64 == 3) {
    // uint8 low bytes (out_mode 4): sixteen entries per lane, one 16-byte store; the first (16 - q0 % 16) % 16
    // entries go alone so that the groups are 16-byte aligned
    if (k == 1u && q0 + nq <= A.cap && ((uintptr_t)A.out & 15u) == 0) {
      uint8_t* o = reinterpret_cast<uint8_t*>(A.out) + q0;
      const uint32_t hh = (uint32_t)((16u - (uint32_t)(q0 & 15u)) & 15u);
      const uint32_t h = hh < nq ? hh : nq;
      if ((uint32_t)lane < h) o[lane] = (uint8_t)(add + ev((uint32_t)lane));
      const uint32_t m = nq - h, g = m >> 4;
      const uint32_t a8 = (uint32_t)add & 0xFFu;
      for (uint32_t t = (uint32_t)lane; t < g; t += kWave) {
        const uint32_t i = h + 16u * t;
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t b0 = (a8 + ev(i + 4u * e)) & 0xFFu, b1 = (a8 + ev(i + 4u * e + 1u)) & 0xFFu;
          const uint32_t b2 = (a8 + ev(i + 4u * e + 2u)) & 0xFFu, b3 = (a8 + ev(i + 4u * e + 3u)) & 0xFFu;
          w[e] = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
        }
        const v4u pk = {w[0], w[1], w[2], w[3]};
        __builtin_nontemporal_store(pk, reinterpret_cast<v4u*>(o + i));
      }
      for (uint32_t t = h + 16u * g + (uint32_t)lane; t < nq; t += kWave) o[t] = (uint8_t)(add + ev(t));
      return false;
    }
  }
  for (uint32_t t = (uint32_t)lane; t < nq; t += kWave) {
    const uint64_t q = q0 + t;
    const uint64_t val = add + ev(r0 + t * k);
    if (near4g) ovf |= val > 0xFFFFFFFFull;
    put<OutT, true>(A.out, q < last ? q : last, val);
  }
  return ovf;
}

// Phase B of one unit on one data wave, once its prefix is set: the event list copied to the output at
// its final index.  FASTA: the list was built under "no header pending at the range start"; if the true
// state S says one is pending, the range's first segment emits nothing (drop its start, fV) and its first
// '\n' ends the pending header (prepend it unless already listed).  Output slot of event i: 2P - S + i
// (u32 slots, starts even, ends odd = '\n' + 1).  Stores go to min(slot, last): an overflowing launch
// reports DP_ERR_CAPACITY and its output is discarded, so the clamp replaces a per-store branch.
template <int MODE, int OUT64>
__device__ __forceinline__ void phase_b(const ScanArgs& A, Shared& sh, uint32_t s, int wave, int lane,
                                        uint32_t& ev_tail) {
  typedef OutOf<OUT64> OutT;
  const WaveRec& rr = sh.rec[s][wave];
  const uint64_t wbase = rfl64(rr.wbase);
  const uint32_t fl = rfl(rr.fl), ev0 = rfl(rr.ev0), nev = rfl(rr.nev);
  const uint64_t P = rfl64(sh.P[s][wave]);
  const uint32_t S = rfl(sh.S[s][wave]);
  ev_tail = ev0 + nev;
  if constexpr (MODE == kDelim && OUT64 >= 2) {
    // uint16 / uint8 low words: the entries before every 64 KiB boundary that starts a wave range (the ranges are
    // split at the first such boundary, so every later one starts a range) locate each entry's block
    // Written only by the range whose chunk holds the boundary byte itself (lo_w == 0, hi_w > 0): a range
    // past the end of a chunk's last unit would write the count at that chunk's end, and the first range of
    // a chunk starting just after the boundary would count bytes of the previous chunk.
    const uint64_t off0 = A.obj_base - A.shift + wbase;
    const uint64_t j = (off0 >> 16) - A.tab_j0;
    const uint32_t lohi = rfl(rr.lohi);
    const bool holds = (lohi & 0xFFFFu) == 0u && (lohi >> 16) != 0u;
    if ((off0 & 0xFFFFull) == 0 && holds && off0 >= (A.tab_j0 << 16) && j < A.tab_n && lane == 0) A.blocktab[j] = P;
  }
  if (fl & kFlDense) {
    dense_b<MODE, OUT64>(A, wbase, rfl(rr.lohi), P, S, lane);
    return;
  }
  const uint64_t obj_off = A.obj_base - A.shift + wbase;
  const bool near4g = OUT64 == 0 && !A.wrap32 && obj_off + kWaveBytes + 1 > 0xFFFFFFFFull;
  const uint16_t* evw = sh.ev[wave];
  bool ovf = false;
  if constexpr (MODE == kFasta) {
    const uint32_t fn = rfl(rr.fn);
    const uint32_t skip = S & (fl >> 2) & 1u;
    const uint32_t pre = (S && !((fl >> 2) & 1u) && fn) ? 1u : 0u;
    const uint32_t n = nev - skip + pre;
    const uint64_t b0 = 2 * P - S, last = 2 * A.cap - 1;
    for (uint32_t i = (uint32_t)lane; i < n; i += kWave) {
      const uint32_t e = (pre && i == 0) ? fn - 1u : (uint32_t)evw[(ev0 + i + skip - pre) & kEvMask];
      const uint64_t slot = b0 + i;
      const uint64_t val = obj_off + e + (slot & 1u);
      if (near4g) ovf |= val > 0xFFFFFFFFull;
      put<OutT>(A.out, slot < last ? slot : last, val);
    }
  } else {
    auto ev = [&](uint32_t i) { return (uint32_t)evw[(ev0 + i) & kEvMask]; };
    ovf = place_delims<OUT64>(A, ev, nev, P, obj_off, lane);
    if constexpr (OUT64 == 3) {
      const uint32_t lohi = rfl(rr.lohi);
      place_subs(A, ev, nev, P, obj_off, (int)(lohi & 0xFFFFu), (int)(lohi >> 16), lane);
    }
  }
  if (ovf) atomicOr(A.err, kErrOverflow);
}

// Bounded LDS poll for a value written by another wave of the workgroup.
__device__ __forceinline__ bool lds_wait_eq(const uint32_t* p, uint32_t v, uint32_t* err) {
  uint64_t t0 = 0;
  for (uint32_t spins = 0; lds_ld(p) != v; ++spins) {
    if (wait_expired(spins, t0)) {
      if (__lane_id() == 0) atomicOr(err, kErrTimeout);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  cbar();
  return true;
}

// The unit's 15 wave summaries composed lane-parallel: lane i < 15 holds wave i, an inclusive DPP scan over
// row 0 gives every wave's exclusive prefix function (lane i-1's inclusive) and the unit's function (lane 15,
// whose own summary is the identity).  Counts of one unit fit 32 bits.
struct Func32 {
  uint32_t cF, cT, sF, sT;
};
__device__ __forceinline__ Func32 f32_then(const Func32& a, const Func32& b) {   // a, then b
  Func32 r;
  r.cF = a.cF + (a.sF ? b.cT : b.cF);
  r.sF = a.sF ? b.sT : b.sF;
  r.cT = a.cT + (a.sT ? b.cT : b.cF);
  r.sT = a.sT ? b.sT : b.sF;
  return r;
}
template <int CTRL, int ROWS>
__device__ __forceinline__ Func32 f32_dpp(const Func32& f) {   // identity where there is no source lane
  return Func32{dpp32<CTRL, ROWS>(f.cF, 0u), dpp32<CTRL, ROWS>(f.cT, 0u), dpp32<CTRL, ROWS>(f.sF, 0u),
                dpp32<CTRL, ROWS>(f.sT, 1u)};
}
__device__ __forceinline__ Func compose_unit(Shared& sh, uint32_t s, int lane) {
  Func32 w = Func32{0, 0, 0, 1};
  if (lane < kDataWaves) {
    const WaveRec& r = sh.rec[s][lane];
    const uint32_t fl = r.fl;
    w = Func32{r.cF, r.cT, fl & 1u, (fl >> 1) & 1u};
  }
  Func32 inc = w;
  inc = f32_then(f32_dpp<kRowShr1, 0xF>(inc), inc);
  inc = f32_then(f32_dpp<kRowShr2, 0xF>(inc), inc);
  inc = f32_then(f32_dpp<kRowShr4, 0xF>(inc), inc);
  inc = f32_then(f32_dpp<kRowShr8, 0xF>(inc), inc);
  const Func32 ex = f32_dpp<kRowShr1, 0xF>(inc);
  if (lane < kDataWaves) {
    sh.exF[s][lane] = ex.cF;
    sh.exT[s][lane] = ex.cT;
    sh.es[s][lane] = (ex.sF & 1u) | ((ex.sT & 1u) << 1);
  }
  const Func unit = Func{(uint32_t)__builtin_amdgcn_readlane((int)inc.cF, kDataWaves),
                         (uint32_t)__builtin_amdgcn_readlane((int)inc.cT, kDataWaves),
                         (uint32_t)__builtin_amdgcn_readlane((int)inc.sF, kDataWaves),
                         (uint32_t)__builtin_amdgcn_readlane((int)inc.sT, kDataWaves)};
  if (lane == 0) {
    sh.uF[s] = (uint32_t)unit.cF;
    sh.uT[s] = (uint32_t)unit.cT;
    sh.us[s] = (unit.sF & 1u) | ((unit.sT & 1u) << 1);
  }
  return unit;
}

// Coordinator issue priority.  At 0 it loses every arbitration to the data waves of its SIMD, which
// (memory permitting) always have an instruction ready: on some XCDs the workgroups' first AGGs came
// ~100 us late (tools/timeline.py; every look-back waits on them), and FASTA is 2-3 % faster at 3.  The
// write-heavy CSV newline index is 4 % slower at 3 (its look-back polls then compete with phase B).
constexpr uint32_t kCoordPrioFasta = 3, kCoordPrioDelim = 0;
constexpr uint32_t kIdleSleep = 1;                 // coordinator back-off (x 64 clocks) after a round without progress
// look-back windows in flight per coordinator attempt: 8 windows (64 VGPRs of descriptors) pushed the
// coordinator path past the kernel's 128 VGPRs and spilled to scratch (44-52 B/lane); 6 spills nothing
// (FASTA +1.4-2.3 % same box, DELIM +-1 %)
constexpr uint32_t kLbDepth = 6;

// consecutive units per ticket atomic: one returning atomic on one address per unit caps the grid near
// 20 units/us (measured: FASTA -16% at 1, -7% at 2, parity at 4); a longer run of consecutive units
// per workgroup delays the next workgroup's look-back, which an event-dense DELIM scan feels first (its
// per-wave event lists fill): CSV (~6,900 delimiters per unit) -20% at 4 vs 2, while VCF (~3,100) and
// FASTQ (~4,300) gain 5% at 4.  DELIM picks the run from the last composed unit's delimiter count.
template <int MODE> constexpr uint32_t kClaimN = MODE == kFasta ? kClaimFasta : kClaimDelimDense;

// Coordinator event loop.  Its descriptor loads queue behind the CU's in-flight input stream (~5 us),
// so it never waits on one unit: each round it issues the look-back windows of up to kLbDepth composed
// units at once, composes + publishes every unit whose 15 data waves are done while they travel (other
// workgroups' look-backs wait on those), then resolves the windows in order until one is incomplete.
template <int MODE>
__device__ __forceinline__ void coordinator(const ScanArgs& A, const Tab& T, int lane, Shared& sh) {
  set_prio(MODE == kFasta ? kCoordPrioFasta : kCoordPrioDelim);
  Cursor cur{0, 0, 0, 0, 0, 0};
  uint64_t prevP = 0;
  uint32_t prevS = 0;
  uint32_t pub = 0, res = 0;
  uint32_t idle = 0;
  uint64_t idle_t0 = 0;
  const uint32_t nunits = (uint32_t)A.nunits;
  uint32_t claimed = 0;                             // steps claimed so far
  uint32_t K = kNoUnit;                             // the workgroup's step count, once a claim ran out of units
  auto unit_of = [&](uint32_t k) { return sh.uq[k % kUnitQ]; };
  // claim units for the steps up to kClaimAhead past the front data wave's (the wave at step k prefetches
  // step k + 1's unit); one returning atomic per unit, on this wave (the data waves' loads are hand-waited)
  uint32_t batch = 0, nbatch = 0;                   // consecutive units of the last claim not yet queued
  uint32_t last_events = ~0u;                       // delimiters of the last composed unit (none yet: dense)
  auto claim_ahead = [&]() {
    bool any = false;
    while (K == kNoUnit && claimed <= lds_ld(&sh.front) + kClaimAhead) {
      if (nbatch == 0) {
        uint32_t u = 0;
        // DELIM: long runs while the units are event-sparse, short ones once a unit is event-dense
        uint32_t run = MODE == kFasta ? kClaimN<MODE> : (last_events > kClaimDense ? kClaimN<MODE> : kClaimDelimSparse);
        // FASTA's first round: one unit per workgroup, so the first prefixes need only the first step's
        // AGGs (FASTA +0.9-2.2 % same box; DELIM -0.4-0.9 %, so it keeps its runs)
        if (MODE == kFasta && claimed == 0) run = 1;
        if (lane == 0) u = atomicAdd(&A.ticket[0], run);
        batch = rfl(u);
        nbatch = run;
      }
      const uint32_t u = batch++;
      --nbatch;
      const uint32_t v = u < nunits ? u : kNoUnit;
      const uint32_t slot = claimed % kUnitQ;
      if (lane == 0) {
        sh.uq[slot] = v;
        cbar();
        lds_st(&sh.uq_ready[slot], claimed + 1u);
      }
      if (v == kNoUnit) K = claimed;
      ++claimed;
      any = true;
    }
    return any;
  };
  auto compose_ready = [&]() {
    bool any = false;
    while (pub < K && lds_ld(&sh.done[pub % kRing]) == (uint32_t)kDataWaves) {
      const uint32_t s = pub % kRing;
      cbar();
      const Func f = compose_unit(sh, s, lane);
      if constexpr (MODE == kDelim) last_events = (uint32_t)f.cF;
      const uint32_t up = unit_of(pub);
      if (lane == 0) {
        if (up > 0) st_desc(&A.desc[up], pack_agg(f) | A.epoch);
        sh.done[s] = 0;                               // slot's counter free for unit pub + kRing
      }
      ++pub;
      any = true;
    }
    return any;
  };
  while (res < K) {
    bool prog = claim_ahead();
    prog |= compose_ready();
    if (res < pub) {
      const uint32_t D = pub - res < kLbDepth ? pub - res : kLbDepth;
      uint64_t d[kLbDepth][kLbPer];
      uint32_t Wj[kLbDepth];
#pragma unroll
      for (uint32_t j = 0; j < kLbDepth; ++j) {
        if (j < D) {
          const uint32_t u = unit_of(res + j);
          Wj[j] = lb_span(u, res + j > 0 ? unit_of(res + j - 1) : kNoUnit);
          lb_load(A, u, Wj[j], lane, d[j]);
        }
      }
      prog |= compose_ready();                        // while the windows travel
#pragma unroll
      for (uint32_t j = 0; j < kLbDepth; ++j) {
        if (j >= D) break;
        const uint32_t u = unit_of(res);
        uint64_t P;
        uint32_t S_in;
        if (!lb_reduce(d[j], Wj[j], pack_prefix(res > 0 ? prevP : 0ull, res > 0 ? prevS : 0u), lane, P, S_in)) {
          break;
        }
        const uint32_t s = res % kRing;
        const Geo g = geo_of(T, (uint32_t)A.nchunks, (uint32_t)A.nunits, u, cur);
        const uint32_t usv = sh.us[s];
        const uint64_t P_incl = P + (S_in ? sh.uT[s] : sh.uF[s]);
        const uint32_t S_out = S_in ? (usv >> 1) & 1u : usv & 1u;
        prevP = P_incl;
        prevS = S_out;
        const uint32_t st0 = (g.fl & kGeoFirst) ? 0u : S_in;
        if (lane < kDataWaves) {                      // per-wave prefixes, one lane per wave
          const uint32_t es = sh.es[s][lane];
          sh.P[s][lane] = P + (st0 ? sh.exT[s][lane] : sh.exF[s][lane]);
          sh.S[s][lane] = st0 ? (es >> 1) & 1u : es & 1u;
        }
        if (lane == 0) {
          st_desc(&A.desc[u], pack_prefix(P_incl, S_out) | A.epoch);
          if (u + 1 == A.nunits) A.total[0] = P_incl;
          if (g.fl & kGeoLast) {
            A.chunk_end[g.c] = P_incl;
            if constexpr (MODE == kFasta) A.pending[g.c] = S_out ? (long long)P_incl - 1 : -1ll;
          }
        }
        // LDS ops of one wave complete in order: every lane's P/S write lands before lane 0's flag
        cbar();
        if (lane == 0) lds_st(&sh.ready[s], res + 1u);
        ++res;
        prog = true;
      }
    }
    if (prog) {
      idle = 0;
      idle_t0 = 0;
    } else {
      if (wait_expired(++idle, idle_t0)) {
        if (lane == 0) atomicOr(A.err, kErrTimeout);
        break;
      }
      __builtin_amdgcn_s_sleep(kIdleSleep);
    }
  }
}

// Data wave: phase A of every unit of the workgroup in order (double-buffered loads two units ahead),
// phase B of each unit as soon as its prefix is ready, waiting only when kRing units or the event list
// would be exceeded.
template <int MODE, int OUT64>
struct DataWave {
  const ScanArgs& A;
  const Tab& T;
  Shared& sh;
  int lane, wave;
  uint32_t ev_head = 0, ev_tail = 0;
  uint32_t jt = 0;                                   // oldest unit whose phase B is not done

  __device__ DataWave(const ScanArgs& a, const Tab& t, Shared& s, int l, int w)
      : A(a), T(t), sh(s), lane(l), wave(w) {}

  // the unit the coordinator claimed for the workgroup's step k (kNoUnit: past the last unit)
  __device__ __forceinline__ uint32_t unit_of(uint32_t k) {
    const uint32_t slot = k % kUnitQ;
    if (!lds_wait_eq(&sh.uq_ready[slot], k + 1u, A.err)) return kNoUnit;
    return rfl(sh.uq[slot]);
  }

  __device__ __forceinline__ void finish(bool block) {
    const uint32_t s = jt % kRing;
    if (block) {
      lds_wait_eq(&sh.ready[s], jt + 1u, A.err);
    }
    phase_b<MODE, OUT64>(A, sh, s, wave, lane, ev_tail);
    ++jt;
  }

  // Unit k: for each buffer h in order, phase A over it, then (but for the last) its prefetch for unit
  // k + 1; publish; phase B of ready units; prefetch of the last buffer.  While one buffer is scanned the
  // kBufs - 1 others are in flight.
  __device__ __forceinline__ bool step(uint32_t k, Geo& g, Buf (&b)[kBufs], Cursor& cur) {
    // sh.front = the workgroup's front step (the coordinator claims units ahead of it)
    uint32_t front = 0;
    if (lane == 0) front = __hip_atomic_fetch_max(&sh.front, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    front = rfl(front);
    // Issue priority = how many units this wave trails the workgroup's front wave (0..3): a unit's AGG
    // waits for its slowest wave, so the trailing waves take issue slots from the leading ones.
    {
      const uint32_t lag = front > k ? front - k : 0u;
      set_prio(lag < 3u ? lag : 3u);
    }
    const uint32_t s = k % kRing;
    wait_buf(b[0]);
    const uint32_t un = unit_of(k + 1u);
    const Geo gn = geo_of(T, (uint32_t)A.nchunks, (uint32_t)A.nunits, un, cur);
    PhaseA pa;
    pa.st = FState{0u, 0u, 0u, -1, 0u, 0u};
    pa.wbase = g.ubase + (uint64_t)wave * kWaveBytes;
    pa.lo = wave_lo(g, wave);
    pa.hi = wave_hi(g, wave);
#pragma unroll
    for (int h = 0; h < kBufs; ++h) {
      if (h > 0) {
        wait_buf(b[h]);                               // this buffer landed; the others stay in flight
      }
      phase_a_half<MODE, OUT64>(A, pa, b[h], h, wave, lane, sh, ev_head);
      if (h + 1 < kBufs) load_buf(b[h], A, gn, wave, lane, h);
    }
    WaveRec rec;
    phase_a_rec<MODE>(pa, g, wave, ev_head, rec);
    ev_head += rec.nev;
    if (lane == 0) {
      sh.rec[s][wave] = rec;
      cbar();
      lds_add(&sh.done[s], 1u);
    }
    // phase B of every unit whose prefix is already there, and (waiting) of the oldest ones until unit
    // k + 1 has a ring slot and kDenseMax free list entries.  Here, between phase A and the last prefetch,
    // the last buffer's registers are free (dense rescans use them).
    while (jt <= k) {
      const bool room = k + 1u - jt < kRing && ev_head - ev_tail <= kEvCap - kDenseMax;
      const bool rdy = lds_ld(&sh.ready[jt % kRing]) == jt + 1u;
      if (!rdy && room) break;
      cbar();
      finish(!rdy);
    }
    load_buf(b[kBufs - 1], A, gn, wave, lane, kBufs - 1);
    g = gn;
    return un < (uint32_t)A.nunits;
  }

  __device__ __forceinline__ void run() {
    Cursor cur{0, 0, 0, 0, 0, 0};
    const uint32_t u0 = unit_of(0);
    if (u0 == kNoUnit) return;                         // every unit was claimed before this workgroup ran
    Geo g = geo_of(T, (uint32_t)A.nchunks, (uint32_t)A.nunits, u0, cur);
    Buf b[kBufs];
#pragma unroll
    for (int h = 0; h < kBufs; ++h) load_buf(b[h], A, g, wave, lane, h);
    uint32_t K = 0;                                    // the workgroup's step count (>= 1: u0 is a unit)
    for (bool more = true; more; ++K) more = step(K, g, b, cur);
    drain_bufs(b);
    while (jt < K) finish(true);         // the tail: wait for the workgroup's last prefixes
  }
};

template <int MODE, int OUT64>
__global__ void __launch_bounds__(kThreads) scan_kernel(ScanArgs A, const uint64_t* __restrict__ tab_lo,
                                                        const uint64_t* __restrict__ tab_hi,
                                                        const uint64_t* __restrict__ tab_u0) {
  if (A.pick != nullptr && *(const cu32s*)(uintptr_t)A.pick != kFormOne) return;   // (uniform) the probe chose line_kernel
  const int lane = __lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __shared__ Shared sh;
  const Tab T{(cu64*)tab_lo, (cu64*)tab_hi, (cu64*)tab_u0};
  const uint32_t G = gridDim.x;
  if (threadIdx.x < kRing) {
    sh.done[threadIdx.x] = 0;
    sh.ready[threadIdx.x] = 0;
  }
  if (threadIdx.x < kUnitQ) sh.uq_ready[threadIdx.x] = 0;
  if (threadIdx.x == 0) sh.front = 0;
  __syncthreads();
  if (wave == kCoord) {
    coordinator<MODE>(A, T, lane, sh);
  } else {
    DataWave<MODE, OUT64> dw(A, T, sh, lane, wave);
    dw.run();
  }
  // every claim of this workgroup is done: the last workgroup to finish resets the claim counters for the
  // next launch on this table (no per-launch memset)
  __syncthreads();
  if (threadIdx.x == 0) {
    if (atomicAdd(&A.ticket[1], 1u) == G - 1u) {
      atomicExch(&A.ticket[0], 0u);
      atomicExch(&A.ticket[1], 0u);
    }
  }
}

// ------------------------------------------------------------------------------------------ FASTA, two kernels
// The FASTA index as a map over 16 KiB ranges followed by a small placement kernel:
//   * fasta_map_kernel: every wave streams its own ranges (r = global wave, + all waves, ...) with no
//     inter-wave or inter-workgroup dependency — the geometry of the plain stream kernel.  Per range it
//     writes a 16-byte summary (the range's header count and line state as a function of the incoming
//     state, as in phase A) and its events (16-bit positions, under "no header pending at the range
//     start") to the range's slot of a spill area.
//   * fasta_place_kernel: one workgroup per block of 1024 range summaries (claimed in order from a
//     ticket) scans them, resolves the block's prefix by a decoupled look-back over block descriptors,
//     and copies every range's events to their final index with the pending-header fix-up of phase B.
//     Ranges with more than kSpillCap events ("dense") are rescanned from the input (dense_b).
// The one-pass kernel pays a fixed ~60 us per launch at its start and tail (its look-back chain couples
// every unit to the grid's slowest); here the map streams like the calibration kernel and the placement
// only touches the summaries (16 B per 16 KiB) and the events.
constexpr uint32_t kSpillCap = 512;                 // events kept per range (1 KiB slot); more = dense
// The spill is word-major: 16-byte word j (events 8j .. 8j + 7) of range r at word index j * nranges + r, so
// the placement's threads (one per range) read word j of consecutive ranges from consecutive addresses, and
// the map's 16 waves of a workgroup (on 16 consecutive ranges in the same step) write adjacent words.
__device__ __forceinline__ uint64_t spill_word(uint32_t j, uint64_t r, uint64_t nranges) { return j * nranges + r; }
constexpr uint32_t kPlaceBlock = 1024;              // range summaries per placement workgroup (one per thread)
constexpr uint32_t kStageBytes = 128u << 10;        // LDS staging of a placement block's output run
constexpr uint32_t kMapWaves = 16;                  // map kernel: 16 data waves per workgroup, one per CU, no coordinator
constexpr uint32_t kRecFirst = 16u, kRecLast = 32u; // range record flags (bits 0-3: sF, sT, fV, dense)
// Map kernel policies (each measured against its alternatives): a workgroup barrier per step (its waves on
// adjacent ranges), groups of 16 ranges claimed from a ticket one per atomic (677-681 us vs 687-689 us per 4 GiB with
// two, profiles/r03/knob_ab/), two steps ahead (step it + 2 has its group by the barrier of step it + 1, where its
// loads are issued).
constexpr uint32_t kMapAhead = 2;

struct MapArgs {
  const uint8_t* base;         // 16-byte aligned; coordinates relative to it
  uint64_t nchunks, nranges;
  uint4* rec;                  // [nranges] 16-byte range records
  uint16_t* spill;             // event positions relative to the range, word-major (spill_word)
  unsigned int* ticket;        // next group to claim; zeroed by the placement kernel
  unsigned int* place_ticket;  // [2] the placement kernel's block ticket, zeroed here
};

// Range r of the chunk table (ranges of kWaveBytes in each chunk's aligned coordinates): the Geo of a
// one-range "unit" (lo_u / hi_u relative to the range, clamped like wave_lo / wave_hi of wave 0).
__device__ __forceinline__ Geo range_geo(const Tab& T, uint32_t nchunks, uint32_t nranges, uint32_t r, Cursor& cur) {
  Geo g;
  if (r >= nranges) {
    g.ubase = 0;
    g.lo_u = g.hi_u = g.c = g.fl = 0;
    return g;
  }
  if (!cur.valid || r < cur.u0 || r >= cur.u1) {
    uint32_t c = 0, cn = nchunks;
    while (cn - c > 1) {                               // a wave's ranges are strided: always a search
      const uint32_t m = (c + cn) >> 1;
      if ((uint32_t)T.u0[m] <= r) c = m; else cn = m;
    }
    cur.c = c;
    cur.u0 = (uint32_t)T.u0[c];
    cur.u1 = (uint32_t)T.u0[c + 1];
    cur.lo = T.lo[c];
    cur.hi = T.hi[c];
    cur.valid = 1;
  }
  g.c = cur.c;
  g.ubase = (cur.lo & ~15ull) + (uint64_t)(r - cur.u0) * (uint64_t)kWaveBytes;
  g.lo_u = cur.lo > g.ubase ? (uint32_t)(cur.lo - g.ubase) : 0u;
  const uint64_t hu = cur.hi - g.ubase;
  g.hi_u = hu < (uint64_t)(kWaveBytes + 16) ? (uint32_t)hu : (uint32_t)(kWaveBytes + 16);
  g.fl = kGeoValid | (r == cur.u0 ? kGeoFirst : 0u) | (r + 1 == cur.u1 ? kGeoLast : 0u);
  return g;
}

// One 16-byte-group returning atomic add, hand-waited like the input loads (inline asm: the compiler adds no
// vmcnt wait for it): issued right after a wait_buf, its result is read after the next one (tools/isa_guard.py
// tracks returning atomics with sc0 as hand-waited destinations).
// Called by every lane of the wave (no divergent branch around it, so the compiler sees the destination
// defined in all lanes and merges nothing into it while the atomic is in flight); only lane 0 executes the
// atomic (exec narrowed inside the asm and restored), and only its value is meaningful: read it with
// readfirstlane once the wait has covered it.
__device__ __forceinline__ uint32_t atomic_add_nowait(unsigned int* p, uint32_t v) {
  uint32_t old;
  uint64_t save;
  asm volatile("s_mov_b64 %1, exec\n\t"
               "s_mov_b64 exec, 1\n\t"
               "global_atomic_add %0, %2, %3, off sc0\n\t"
               "s_mov_b64 exec, %1"
               : "=&v"(old), "=&s"(save) : "v"(p), "v"(v) : "memory");
  return old;
}

// the same from the chunk table: range r of chunk c (range_geo without the search; FASTA's 16-byte records carry no
// geometry: the placement derives it, which halved the map's record stores, profiles/r04/ab/rec16)
__device__ __forceinline__ uint4 range_geo_rec_tab(const Tab& T, uint32_t c, uint64_t r) {
  const uint64_t lo = T.lo[c], hi = T.hi[c], u0 = T.u0[c];
  const uint64_t ub = (lo & ~15ull) + (r - u0) * (uint64_t)kWaveBytes;
  const uint32_t lo_u = lo > ub ? (uint32_t)(lo - ub) : 0u;
  const uint64_t hu = hi - ub;
  const uint32_t hi_u = hu < (uint64_t)(kWaveBytes + 16) ? (uint32_t)hu : (uint32_t)(kWaveBytes + 16);
  return uint4{(uint32_t)ub, (uint32_t)(ub >> 32), lo_u | (hi_u << 16), 0u};
}
// FASTA range record r's summary word

__global__ void __launch_bounds__(kWave * kMapWaves, 4) map_kernel(MapArgs M, const uint64_t* __restrict__ tab_lo,
                                                                const uint64_t* __restrict__ tab_hi,
                                                                const uint64_t* __restrict__ tab_r0) {
  __shared__ __attribute__((aligned(16))) uint16_t sev[kMapWaves][kSpillCap];
  const int lane = __lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Tab T{(cu64*)tab_lo, (cu64*)tab_hi, (cu64*)tab_r0};
  const uint32_t nranges = (uint32_t)M.nranges, nchunks = (uint32_t)M.nchunks;
  constexpr uint32_t kNwValid = 0x80000000u;
  // every range's record and first kDeferW spill words stay in LDS, kDeferG groups deep, and the workgroup stores
  // them in one burst when the buffer is full and once at the end (its last loads drained): the map's scattered
  // stores inside the read stream cost far more than their bytes (DESIGN.md §4, 644-650 vs 658-662 us)
  constexpr uint32_t kDeferG = 72u, kDeferW = 4u;
  __shared__ uint4 dq_rec[kDeferG][kMapWaves];
  __shared__ uint4 dq_sp[kDeferG][kDeferW][kMapWaves];
  __shared__ uint32_t dq_nw[kDeferG][kMapWaves];      // words buffered | kNwValid (0: no record)
  __shared__ uint32_t dq_r0[kDeferG];
  uint32_t nbuf = 0;                                  // groups buffered (uniform)
  // (every thread, after a barrier) the buffered groups to HBM: per group its 16 records (256 contiguous bytes)
  // and each buffered spill word index (word-major: 256 contiguous bytes)
  auto flush = [&]() {
    constexpr uint32_t kPer = 16u * (1u + kDeferW);
    for (uint32_t e = threadIdx.x; e < nbuf * kPer; e += kWave * kMapWaves) {
      const uint32_t gq = e / kPer, rem = e - gq * kPer, part = rem >> 4, w = rem & 15u;
      const uint32_t nw = dq_nw[gq][w];
      if (!(nw & kNwValid)) continue;
      const uint64_t rr = (uint64_t)dq_r0[gq] + w;
      if (part == 0u) M.rec[rr] = dq_rec[gq][w];
      else if (part - 1u < (nw & 0xFFu))
        reinterpret_cast<v4u*>(M.spill)[spill_word(part - 1u, rr, M.nranges)] =
            *reinterpret_cast<const v4u*>(&dq_sp[gq][part - 1u][w]);
    }
    nbuf = 0;
  };
  // the placement kernel that follows claims its blocks from this ticket: it starts from zero (no memset
  // launch, no end-of-kernel counter; the placement kernel zeroes this kernel's own ticket in turn)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    M.place_ticket[0] = 0u;
    M.place_ticket[1] = 0u;
  }
#ifdef DP_DIAG
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  uint32_t n_done = 0;
#endif
  // Groups of 16 consecutive ranges (one per wave), claimed from a ticket by wave 0 (so faster CUs and XCDs take
  // more groups); s_grp[k % kGrpQ] = the group of step k.
  constexpr uint32_t kGrpQ = 8;
  __shared__ uint32_t s_grp[kGrpQ];
  const uint32_t ngroups = (nranges + kMapWaves - 1) / kMapWaves;
  const uint32_t G = gridDim.x;
  // The first two steps are static (groups blockIdx.x and G + blockIdx.x), so the first loads go out at once;
  // the ticket hands out groups from 2G on, its first claim issued in step 0 like every later one.  Static
  // groups are safe here, and only here, because nothing in this kernel waits on another workgroup: a workgroup
  // that has not started yet delays no one (line_kernel, whose groups wait on their predecessors' counts, claims
  // every group from its ticket: with static first groups two processes' grids sharing a GPU deadlocked, round 4).
  uint32_t claimed = 2, pend = 0;                    // wave 0: steps with a group; the pending claim's size
  uint32_t claim_res = 0;
  if (threadIdx.x == 0) {
    s_grp[0] = blockIdx.x;
    s_grp[1] = G + blockIdx.x;
  }
  __syncthreads();
  // (the host launches at most one workgroup per group, so s_grp[0] = blockIdx.x < ngroups)
  uint32_t r = s_grp[0] * kMapWaves + (uint32_t)wave;
  Cursor cur{0, 0, 0, 0, 0, 0};
  Geo g = range_geo(T, nchunks, nranges, r, cur);
  ScanArgs SA{};                                     // the input loads' base (the map kernel needs nothing else of it)
  SA.base = M.base;
  BufN b[kBufs];
#pragma unroll
  for (int h = 0; h < kBufs; ++h) load_bufx(b[h], SA, g, lane, h);
  for (uint32_t it = 0;; ++it) {
    __syncthreads();
    const uint32_t gnext = s_grp[(it + 1) % kGrpQ];
    const uint32_t rn = gnext < ngroups ? gnext * kMapWaves + (uint32_t)wave : nranges;
    // wave 0 keeps two steps claimed ahead: step it + 2 needs its group by the barrier of step it + 1
    const bool do_claim = wave == 0 && claimed < it + 1u + kMapAhead && s_grp[(claimed - 1) % kGrpQ] < ngroups;
    const Geo gn = range_geo(T, nchunks, nranges, rn, cur);
    FState st{0u, 0u, 0u, -1, 0u, 0u};
    const int lo = (int)g.lo_u, hi = (int)g.hi_u;
    const bool interior = lo == 0 && hi > kWaveBytes;   // wave-uniform
    uint16_t* evw = sev[wave];
    auto keep = [&](uint32_t rk, uint32_t pos) { evw[rk < kSpillCap - 1u ? rk : kSpillCap - 1u] = (uint16_t)pos; };
#pragma unroll
    for (int h = 0; h < kBufs; ++h) {
      wait_bufx(b[h]);                                // this buffer landed; the other stays in flight
      if (h == 0 && do_claim) {                       // the youngest vector-memory operation until the next wait
        claim_res = atomic_add_nowait(M.ticket, 1u);
        pend = 1u;
      }
      if (h == kBufs - 1 && pend) {                   // the wait above covered the claim: its value is back
        asm volatile("" : "+v"(claim_res) :: "memory");
        const uint32_t u = 2u * G + rfl(claim_res);
        if (lane == 0)
          for (uint32_t i = 0; i < pend; ++i) s_grp[(claimed + i) % kGrpQ] = u + i;
        claimed += pend;
        pend = 0;
      }
      v4u x[kRows];
#pragma unroll
      for (int i = 0; i < kRows; ++i) x[i] = b[h].x[i];
      const uint32_t la = lookahead_s(M.base, g, h, interior, hi);
      if (interior) fasta_rows<true>(x, la, h, lo, hi, lane, st, keep);
      else fasta_rows<false>(x, la, h, lo, hi, lane, st, keep);
      if (h + 1 < kBufs) load_bufx(b[h], SA, gn, lane, h);
    }
    const bool dense = st.nev > kSpillCap;
    const uint32_t n = dense ? 0u : st.nev;
    cbar();
    {
      // the range's summary (phase_a_rec of a one-range unit) and its first events to the LDS burst buffer
      if (!st.nlseen) st.fV = st.S;
      uint32_t cT = st.cnt - st.fV, sT = st.nlseen ? st.S : 1u;
      if (g.fl & kGeoFirst) { cT = st.cnt; sT = st.S; }  // chunk start: the incoming state is reset
      const bool valid = (g.fl & kGeoValid) != 0u;
      const uint32_t nwords = (n + 7u) >> 3;
      if (lane == 0) {
        const uint32_t fl = st.S | (sT << 1) | (st.fV << 2) | (dense ? kFlDense : 0u) |
                            ((g.fl & kGeoFirst) ? kRecFirst : 0u) | ((g.fl & kGeoLast) ? kRecLast : 0u);
        dq_nw[nbuf][wave] = valid ? ((nwords < kDeferW ? nwords : kDeferW) | kNwValid) : 0u;
        dq_rec[nbuf][wave] = uint4{st.cnt | (cT << 16), (uint32_t)(st.fn + 1) | (st.nev << 16), fl, g.c};
        if (wave == 0) dq_r0[nbuf] = r;                // (wave 0's range is the group's first)
      }
      if (valid && (uint32_t)lane < nwords) {
        const v4u v = *reinterpret_cast<const v4u*>(evw + lane * 8);
        if ((uint32_t)lane < kDeferW) *reinterpret_cast<v4u*>(&dq_sp[nbuf][lane][wave]) = v;
        else reinterpret_cast<v4u*>(M.spill)[spill_word((uint32_t)lane, r, M.nranges)] = v;   // a rare long list
      }
      if (++nbuf == kDeferG) {                        // uniform: the buffer is full
        __syncthreads();
        flush();
      }
    }
    load_bufx(b[kBufs - 1], SA, gn, lane, kBufs - 1);
#ifdef DP_DIAG
    n_done += (g.fl & kGeoValid) ? 1u : 0u;
#endif
    if (gnext >= ngroups) break;                      // uniform (LDS value read after the barrier)
    r = rn;
    g = gn;
  }
  drain_bufsx(b);
  __syncthreads();                                    // the last buffered groups, after the last loads
  flush();
#ifdef DP_DIAG
  // per wave: start and end (100 MHz realtime clock), ranges scanned, the XCC it ran on
  if (lane == 0 && blockIdx.x < kProfMaxGrid) {
    unsigned long long* w = g_prof + ((uint64_t)blockIdx.x * kProfWaves + wave) * kProfSlots;
    w[0] = t_start;
    w[1] = __builtin_amdgcn_s_memrealtime();
    w[2] = n_done;
    w[3] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) & 0xFu;   // HW_REG_XCC_ID
  }
#endif
}

// Wave-wide (64-lane) inclusive scan of range functions, lane 0 farthest.
__device__ __forceinline__ Func32 f32_wave_scan(Func32 f) {
  f = f32_then(f32_dpp<kRowShr1, 0xF>(f), f);
  f = f32_then(f32_dpp<kRowShr2, 0xF>(f), f);
  f = f32_then(f32_dpp<kRowShr4, 0xF>(f), f);
  f = f32_then(f32_dpp<kRowShr8, 0xF>(f), f);
  f = f32_then(f32_dpp<kRowBcast15, 0xA>(f), f);
  f = f32_then(f32_dpp<kRowBcast31, 0xC>(f), f);
  return f;
}

struct PlaceArgs {
  const uint4* rec;
  const uint16_t* spill;
  uint64_t nranges, nblocks;
  int count_only;              // no output buffer: counts, chunk ends and pending only
  int in_order;                // blocks by blockIdx (nblocks <= kLbSlots), else claimed from the ticket
  unsigned int* map_ticket;    // the map kernel's group ticket, zeroed here for the next launch
};

// (in-order placement) look-back polls before the unpublished AGGs of a window are recomputed from the records
constexpr uint32_t kPlacePolls = 4;
// The AGG descriptor of placement block p from its range records (one wave: 16 consecutive records per lane,
// composed in order, then the wave's inclusive scan), as the block itself publishes it.
__device__ __forceinline__ uint64_t block_agg_from_records(const PlaceArgs& PA, const ScanArgs& A, uint32_t p, int lane) {
  constexpr uint32_t kPer = kPlaceBlock / kWave;
  const uint64_t r0 = (uint64_t)p * kPlaceBlock + (uint64_t)lane * kPer;
  uint4 rc[kPer];
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) rc[i] = r0 + i < PA.nranges ? PA.rec[r0 + i] : uint4{0u, 0u, 2u, 0u};
  Func32 f{0u, 0u, 0u, 1u};
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i)
    f = f32_then(f, Func32{rc[i].x & 0xFFFFu, rc[i].x >> 16, rc[i].z & 1u, (rc[i].z >> 1) & 1u});
  const Func32 w = f32_wave_scan(f);
  const Func agg{(uint32_t)__builtin_amdgcn_readlane((int)w.cF, kWave - 1), (uint32_t)__builtin_amdgcn_readlane((int)w.cT, kWave - 1),
                 (uint32_t)__builtin_amdgcn_readlane((int)w.sF, kWave - 1) & 1u,
                 (uint32_t)__builtin_amdgcn_readlane((int)w.sT, kWave - 1) & 1u};
  return pack_agg(agg) | A.epoch;
}

// Every slot of a loaded look-back window of block b whose descriptor is unpublished gets that block's AGG,
// recomputed from its records (one block at a time, the whole wave).
__device__ __forceinline__ void lb_fill_from_records(const PlaceArgs& PA, const ScanArgs& A, uint32_t b, uint32_t W,
                                                     int lane, uint64_t (&d)[kLbPer]) {
  const uint32_t rl = (uint32_t)(kWave - 1 - lane);
  for (;;) {
    uint32_t mine = kLbPer;
#pragma unroll
    for (int j = kLbPer - 1; j >= 0; --j) {
      const uint32_t k = kLbPer * rl + (uint32_t)j;
      if (k < W && (d[j] & kStatMask) == 0ull) mine = (uint32_t)j;
    }
    const uint64_t bal = __ballot(mine < kLbPer);
    if (bal == 0ull) return;
    const int L = 63 - __builtin_clzll(bal);
    const uint32_t j = (uint32_t)__builtin_amdgcn_readlane((int)mine, L);
    const uint32_t k = kLbPer * (uint32_t)(kWave - 1 - L) + j;
    const uint64_t agg = block_agg_from_records(PA, A, b - 1u - k, lane);
#pragma unroll
    for (int jj = 0; jj < kLbPer; ++jj)
      if (lane == L && (uint32_t)jj == j) d[jj] = agg;
  }
}

// LDS of one placement block
struct PlaceShared {
  Func32 wagg[kPlaceBlock / kWave];
  Func32 wex[kPlaceBlock / kWave];
  uint64_t P;
  uint32_t S, ndense, anydense, blk;
  unsigned long long lo, hi;                          // the block's output run
  uint32_t dense[kPlaceBlock];
  uint64_t dP[kPlaceBlock];
  uint32_t dS[kPlaceBlock];
  // the block's output slots are one contiguous run: staged here, then written with coalesced 16-byte stores
  uint4 stage[kStageBytes / 16];
};

// One placement block b (1024 range records): every thread of the workgroup takes part; ends with a barrier,
// so the caller may reuse `ps` at once.
template <int OUT64>
__device__ __forceinline__ void fasta_place_block(const PlaceArgs& PA, const ScanArgs& A, const Tab& T, uint32_t b,
                                                  PlaceShared& ps) {
  typedef typename std::conditional<OUT64 == 1, uint64_t, uint32_t>::type OutT;
  constexpr int kPW = kPlaceBlock / kWave;           // 16 waves
  const int lane = __lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  OutT* s_stage = reinterpret_cast<OutT*>(ps.stage);
  if (threadIdx.x == 0) {
    ps.ndense = 0;
    ps.lo = 0;
    ps.hi = 0;
    ps.anydense = 0;
  }
  __syncthreads();
#ifdef DP_DIAG
  // per block (diagnostics build): realtime stamps at its sections, in g_prof past the map kernel's words
  unsigned long long* pst = g_prof + ((uint64_t)(512u + (b & 511u)) * kProfWaves) * kProfSlots;
#define PLACE_STAMP(i) do { if (threadIdx.x == 0 && b < 512u) pst[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define PLACE_STAMP(i) do {} while (0)
#endif
  PLACE_STAMP(0);
  const uint64_t r = (uint64_t)b * kPlaceBlock + threadIdx.x;
  const bool valid = r < PA.nranges;
  uint4 rc = uint4{0u, 0u, 2u, 0u};                   // identity: no count, state kept
  uint4 rg = uint4{0u, 0u, 0u, 0u};
  if (valid) {
    rc = PA.rec[r];
    rg = range_geo_rec_tab(T, rc.w, r);
  }
  const uint32_t cF = rc.x & 0xFFFFu, cT = rc.x >> 16, fl = rc.z;
  // what the placement needs besides the prefix is loaded now, under the scan and the look-back: the
  // range's first four spill words (32 events).  With two (16 events), a quarter of the configs[1] ranges
  // (8 headers per 16 KiB, up to 11) needed a third word after the prefix, i.e. one more dependent load in
  // every block.
  const uint32_t nev = rc.y >> 16;
  const uint64_t wbase = (uint64_t)rg.x | ((uint64_t)rg.y << 32);
  uint4 sw0 = uint4{0u, 0u, 0u, 0u}, sw1 = sw0, sw2 = sw0, sw3 = sw0;
  const uint4* sp = reinterpret_cast<const uint4*>(PA.spill);
  if (valid && !PA.count_only) {
    if (!(fl & kFlDense)) {
      if (nev > 0u) sw0 = sp[spill_word(0u, r, PA.nranges)];
      if (nev > 8u) sw1 = sp[spill_word(1u, r, PA.nranges)];
      if (nev > 16u) sw2 = sp[spill_word(2u, r, PA.nranges)];
      if (nev > 24u) sw3 = sp[spill_word(3u, r, PA.nranges)];
    }
  }
  const Func32 f{cF, cT, fl & 1u, (fl >> 1) & 1u};
  const Func32 inc = f32_wave_scan(f);
  const Func32 ex = Func32{dpp32<kWaveShr1, 0xF>(inc.cF, 0u), dpp32<kWaveShr1, 0xF>(inc.cT, 0u),
                           dpp32<kWaveShr1, 0xF>(inc.sF, 0u), dpp32<kWaveShr1, 0xF>(inc.sT, 1u)};
  if (lane == kWave - 1) ps.wagg[wave] = inc;
  PLACE_STAMP(1);
  __syncthreads();
  if (wave == 0) {
    Func32 w = lane < kPW ? ps.wagg[lane] : Func32{0, 0, 0, 1};
    Func32 wi = w;
    wi = f32_then(f32_dpp<kRowShr1, 0xF>(wi), wi);
    wi = f32_then(f32_dpp<kRowShr2, 0xF>(wi), wi);
    wi = f32_then(f32_dpp<kRowShr4, 0xF>(wi), wi);
    wi = f32_then(f32_dpp<kRowShr8, 0xF>(wi), wi);
    const Func32 we = f32_dpp<kRowShr1, 0xF>(wi);
    if (lane < kPW) ps.wex[lane] = we;
    const Func agg{(uint32_t)__builtin_amdgcn_readlane((int)wi.cF, kPW - 1),
                   (uint32_t)__builtin_amdgcn_readlane((int)wi.cT, kPW - 1),
                   (uint32_t)__builtin_amdgcn_readlane((int)wi.sF, kPW - 1) & 1u,
                   (uint32_t)__builtin_amdgcn_readlane((int)wi.sT, kPW - 1) & 1u};
    // the block's exclusive prefix: a decoupled look-back over the block descriptors
    uint64_t P = 0;
    uint32_t S = 0;
    PLACE_STAMP(2);
    if (b > 0) {
      if (lane == 0) st_desc(&A.desc[b], pack_agg(agg) | A.epoch);
      const uint32_t W = lb_span(b, kNoUnit);
      uint64_t t0 = 0;
      for (uint32_t spins = 0;; ++spins) {
        uint64_t d[kLbPer];
        lb_load(A, b, W, lane, d);
        if (lb_reduce(d, W, pack_prefix(0ull, 0u), lane, P, S)) break;
        if (PA.in_order && spins >= kPlacePolls) {
          // (blocks by blockIdx) never wait on a block that may not be running: the AGG of every predecessor
          // still unpublished is recomputed from its records, and the window (which reaches the base: b <
          // kLbSlots) then resolves
          lb_fill_from_records(PA, A, b, W, lane, d);
          if (lb_reduce(d, W, pack_prefix(0ull, 0u), lane, P, S)) break;
        }
        if (wait_expired(spins, t0)) {
          if (lane == 0) atomicOr(A.err, kErrTimeout);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    const uint64_t P_incl = P + (S ? agg.cT : agg.cF);
    const uint32_t S_out = S ? agg.sT : agg.sF;
    if (lane == 0) {
      st_desc(&A.desc[b], pack_prefix(P_incl, S_out) | A.epoch);
      ps.P = P;
      ps.S = S;
    }
    PLACE_STAMP(3);
  }
  __syncthreads();
  const uint64_t Pb = ps.P;
  const uint32_t Sb = ps.S;
  // this range's incoming state: the block prefix, then the waves before it, then the lanes before it
  const Func32 wx = ps.wex[wave];
  const uint64_t Pw = Pb + (Sb ? wx.cT : wx.cF);
  const uint32_t Sw = Sb ? wx.sT : wx.sF;
  uint64_t P = Pw + (Sw ? ex.cT : ex.cF);
  uint32_t S = (Sw ? ex.sT : ex.sF) & 1u;
  if (fl & kRecFirst) S = 0u;                         // chunk start: no header pending
  // this range's output run: slots [b0, b0 + n) (the fix-up of phase_b: drop a start pending from the
  // previous range, prepend the end of the header pending into it)
  const uint32_t fn = rc.y & 0xFFFFu;
  const uint32_t fV = (fl >> 2) & 1u;
  const uint32_t skip = S & fV;
  const uint32_t pre = (S && !fV && fn) ? 1u : 0u;
  const uint64_t b0 = 2 * P - S;
  // the ranges' runs follow one another in range order: the block's run is [b0 of its first range, end of its
  // last); a dense range (its count of slots is not in the record) means no staging
  if (valid && !PA.count_only) {
    if (fl & kFlDense) ps.anydense = 1u;
    if (threadIdx.x == 0) ps.lo = b0;
    if (r + 1 == PA.nranges || threadIdx.x == kPlaceBlock - 1) ps.hi = b0 + nev - skip + pre;
  }
  __syncthreads();
  PLACE_STAMP(7);
  const uint64_t last = 2 * A.cap - 1;
  const uint64_t run_lo = ps.lo, run_hi = ps.hi < last + 1 ? ps.hi : last + 1;
  constexpr uint32_t kVec = 16u / sizeof(OutT);
  const uint64_t stage0 = run_lo & ~(uint64_t)(kVec - 1u);
  const bool stage = !PA.count_only && !ps.anydense && run_lo < run_hi &&
                     (run_hi - stage0) * sizeof(OutT) <= kStageBytes;
  if (valid && !PA.count_only) {
    if (fl & kFlDense) {
      ps.dense[atomicAdd(&ps.ndense, 1u)] = threadIdx.x;
    } else {
      const uint64_t obj_off = A.obj_base - A.shift + wbase;
      const bool near4g = OUT64 == 0 && obj_off + kWaveBytes + 1 > 0xFFFFFFFFull;
      bool ovf = false;
      auto emit = [&](uint64_t slot, uint32_t e) {
        const uint64_t val = obj_off + e + (slot & 1u);
        if (near4g) ovf |= val > 0xFFFFFFFFull;
        if (stage) {
          if (slot <= last) s_stage[(uint32_t)(slot - stage0)] = (OutT)val;
        } else {
          put<OutT>(A.out, slot < last ? slot : last, val);
        }
      };
      if (pre) emit(b0, fn - 1u);
      const uint64_t base_slot = b0 + pre - skip;     // event k goes to base_slot + k (k >= skip)
      // (the prefetched words by name: selecting among them by index made the compiler keep them in a
      // private array in scratch, waiting for their loads at once)
      if (stage && !near4g) {
        // the common case in 32-bit index arithmetic: event k -> s_stage[sb + k] (sb wraps to -1 when the
        // run starts with a skipped event: k >= skip keeps the index in range), its value obj_off + e + the
        // parity of its slot (start or end), slots past the capacity dropped by one bound on k
        const uint32_t sb = (uint32_t)(base_slot - stage0);
        const uint64_t room = last + 1u > base_slot ? last + 1u - base_slot : 0u;
        const uint32_t lim = room < (uint64_t)nev ? (uint32_t)room : nev;
        const OutT o0 = (OutT)obj_off;
        const uint32_t par = (uint32_t)base_slot & 1u;
        auto emit8s = [&](const uint4& v, uint32_t k0) {
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (uint32_t e = 0; e < 8u; ++e) {
            const uint32_t k = k0 + e;
            const uint32_t ev = (w[e >> 1] >> (16u * (e & 1u))) & 0xFFFFu;
            if (k >= skip && k < lim) s_stage[sb + k] = o0 + (OutT)(ev + (par ^ (e & 1u)));
          }
        };
        if (nev > 0u) emit8s(sw0, 0u);
        if (nev > 8u) emit8s(sw1, 8u);
        if (nev > 16u) emit8s(sw2, 16u);
        if (nev > 24u) emit8s(sw3, 24u);
        for (uint32_t k0 = 32u; k0 < nev; k0 += 8u) emit8s(sp[spill_word(k0 >> 3, r, PA.nranges)], k0);
      } else {
        auto emit8 = [&](const uint4& v, uint32_t k0) {
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (uint32_t e = 0; e < 8u; ++e) {
            const uint32_t k = k0 + e;
            if (k >= skip && k < nev) emit(base_slot + k, (w[e >> 1] >> (16u * (e & 1u))) & 0xFFFFu);
          }
        };
        if (nev > 0u) emit8(sw0, 0u);
        if (nev > 8u) emit8(sw1, 8u);
        if (nev > 16u) emit8(sw2, 16u);
        if (nev > 24u) emit8(sw3, 24u);
        for (uint32_t k0 = 32u; k0 < nev; k0 += 8u) emit8(sp[spill_word(k0 >> 3, r, PA.nranges)], k0);
      }
      if (ovf) atomicOr(A.err, kErrOverflow);
    }
  }
  __syncthreads();
  PLACE_STAMP(4);
  if (stage) {
    // coalesced copy of the run; its first and last partial 16-byte groups element by element, so that the
    // neighbouring blocks' slots are never written.  (A header still pending at a chunk end leaves its end
    // slot unwritten here: the resolve kernel, or the host, writes it afterwards.)
    OutT* o = reinterpret_cast<OutT*>(A.out);
    const uint64_t v0 = (run_lo + kVec - 1u) & ~(uint64_t)(kVec - 1u), v1 = run_hi & ~(uint64_t)(kVec - 1u);
    if (v0 <= v1) {
      for (uint64_t q = run_lo + threadIdx.x; q < v0; q += kPlaceBlock) o[q] = s_stage[(uint32_t)(q - stage0)];
      for (uint64_t q = v1 + threadIdx.x; q < run_hi; q += kPlaceBlock) o[q] = s_stage[(uint32_t)(q - stage0)];
      const v4u* src = reinterpret_cast<const v4u*>(s_stage);
      const uint32_t g0 = (uint32_t)((v0 - stage0) / kVec);
      v4u* dst = reinterpret_cast<v4u*>(o + v0);
      for (uint64_t g = threadIdx.x; g < (v1 - v0) / kVec; g += kPlaceBlock) dst[g] = src[g0 + (uint32_t)g];
    } else {                                          // the run lies inside one 16-byte group
      for (uint64_t q = run_lo + threadIdx.x; q < run_hi; q += kPlaceBlock) o[q] = s_stage[(uint32_t)(q - stage0)];
    }
  }
  PLACE_STAMP(5);
  // per-chunk results, after the output stores (a store here would make the loops above wait for it)
  if (valid) {
    const uint64_t P_incl = P + (S ? cT : cF);
    const uint32_t S_out = S ? (fl >> 1) & 1u : fl & 1u;
    if (fl & kRecLast) {
      A.chunk_end[rc.w] = P_incl;
      A.pending[rc.w] = S_out ? (long long)P_incl - 1 : -1ll;
    }
    if (r + 1 == PA.nranges) A.total[0] = P_incl;
  }
  // dense ranges: one wave each, rescanned from the input with the now known state
  const uint32_t nd = ps.ndense;
  if (nd) {
    // every thread keeps its own (P, S); a wave fetches a dense range's through LDS
    ps.dP[threadIdx.x] = P;
    ps.dS[threadIdx.x] = S;
    __syncthreads();
    for (uint32_t i = (uint32_t)wave; i < nd; i += kPW) {
      const uint32_t t = ps.dense[i];
      const uint64_t rr = (uint64_t)b * kPlaceBlock + t;
      const uint4 rq = range_geo_rec_tab(T, PA.rec[rr].w, rr);
      dense_b<kFasta, OUT64>(A, (uint64_t)rq.x | ((uint64_t)rq.y << 32), rq.z, ps.dP[t], ps.dS[t], lane);
    }
  }
  PLACE_STAMP(6);
#undef PLACE_STAMP
  __syncthreads();
}

template <int OUT64>
__global__ void __launch_bounds__(kPlaceBlock) fasta_place_kernel(PlaceArgs PA, ScanArgs A,
                                                                 const uint64_t* __restrict__ tab_lo,
                                                                 const uint64_t* __restrict__ tab_hi,
                                                                 const uint64_t* __restrict__ tab_r0) {
  __shared__ PlaceShared ps;
  if (threadIdx.x == 0) {
    if (blockIdx.x == 0) PA.map_ticket[0] = 0u;       // the map kernel is done with it: ready for the next launch
    // in order (at most kLbSlots blocks): block = blockIdx, no claim (the claims' atomics serialized ~3 us of
    // block starts at 256 blocks); its look-back never waits on a predecessor that is not running (it
    // recomputes such an AGG from the records).  Larger launches claim in order from the ticket: a block only
    // waits on lower, already running or finished, blocks.
    ps.blk = PA.in_order ? blockIdx.x : atomicAdd(&A.ticket[0], 1u);
  }
  __syncthreads();
  const Tab T{(cu64*)tab_lo, (cu64*)tab_hi, (cu64*)tab_r0};
  fasta_place_block<OUT64>(PA, A, T, ps.blk, ps);
}

// ------------------------------------------------------------------------------------------ count look-back
// Look-back over count descriptors (the newline index's groups: an AGG or PREFIX descriptor holds a 48-bit count).
__device__ __forceinline__ uint64_t pack_count(uint64_t st, uint64_t count) { return st | (count & 0xFFFFFFFFFFFFull); }
// the 64-bit sum over the wave (two 32-bit halves through DPP), uniform
__device__ __forceinline__ uint64_t wave_sum64(uint64_t sum) {
  sum += dpp64<kRowShr1, 0xF>(sum, 0ull);
  sum += dpp64<kRowShr2, 0xF>(sum, 0ull);
  sum += dpp64<kRowShr4, 0xF>(sum, 0ull);
  sum += dpp64<kRowShr8, 0xF>(sum, 0ull);
  sum += dpp64<kRowBcast15, 0xA>(sum, 0ull);
  sum += dpp64<kRowBcast31, 0xC>(sum, 0ull);
  return readlane64(sum, kWave - 1);
}
// ``all`` (optional): set, with P = the window's total count, when every descriptor is published and none is a
// PREFIX (the look-back can go on past the window)
__device__ __forceinline__ bool lb_reduce_count(uint64_t (&d)[kLbPer], uint32_t W, uint64_t basedesc, int lane, uint64_t& P,
                                                bool* all = nullptr) {
  const uint32_t rl = (uint32_t)(kWave - 1 - lane);
  uint32_t seen = 0, bad = 0;
#pragma unroll
  for (int j = 0; j < kLbPer; ++j) {                // nearest first
    if (kLbPer * rl + j == W) d[j] = basedesc;
    const uint64_t st = d[j] & kStatMask;
    if (!seen && st == 0ull) bad = 1;
    if (st == kStatPrefix) seen = 1;
  }
  const uint64_t PB = __ballot(seen);
  const uint64_t BB = __ballot(bad);
  if (PB == 0ull) {
    if (all != nullptr && BB == 0ull) {
      uint64_t s = 0;
#pragma unroll
      for (int j = 0; j < kLbPer; ++j) s += d[j] & 0xFFFFFFFFFFFFull;
      P = wave_sum64(s);
      *all = true;
    }
    return false;
  }
  const int Lp = 63 - __builtin_clzll(PB);            // nearest lane holding a prefix
  const uint64_t need = ~((1ull << Lp) - 1ull);
  if (BB & need) return false;
  uint32_t jp = kLbPer;
#pragma unroll
  for (int j = kLbPer - 1; j >= 0; --j)
    if ((d[j] & kStatMask) == kStatPrefix) jp = (uint32_t)j;
  const uint32_t kP = (uint32_t)kLbPer * (uint32_t)(63 - Lp) + (uint32_t)__builtin_amdgcn_readlane((int)jp, Lp);
  uint64_t sum = 0, pv = 0;
#pragma unroll
  for (int j = 0; j < kLbPer; ++j) {
    const uint32_t k = kLbPer * rl + j;
    if (k < kP) sum += d[j] & 0xFFFFFFFFFFFFull;
    if (k == kP) pv = d[j] & 0xFFFFFFFFFFFFull;
  }
  P = readlane64(pv, Lp) + wave_sum64(sum);
  return true;
}

// ------------------------------------------------------------------------------------------ DELIM, lockstep one pass
// line_kernel<OUT64>: the newline index in ONE kernel with the map kernel's geometry (round 4).  A workgroup of
// 16 waves scans a group of 16 consecutive 16 KiB ranges per step (claimed from a ticket, a barrier per step,
// exactly the FASTA map_kernel's streaming loop), but keeps each range's delimiter positions in LDS instead of
// spilling them to HBM, and places them itself once the group's prefix is known:
//   * step k: phase A of group g_k -> LDS slot k % kLineSlots (positions, count, geometry per wave);
//   * step k + 1: wave 0 publishes g_k's delimiter count as an AGG descriptor right after the barrier (every
//     wave wrote its count before it), and at the step's end loads the look-back window of its oldest
//     unresolved group (group descriptors, by LDS-DMA: no VGPR held in flight);
//   * step k + 2: wave 0 reduces that window after its second buffer wait (no stall); a resolved group gets its
//     PREFIX descriptor, every range's launch prefix in LDS and the slot's `res` tag; after their rows, the
//     waves claim the resolved step's 16 ranges from an LDS counter and copy each range's positions to their
//     final index (place_delims), so the waves that finish first place most of them.
// A wave only blocks when the slot it is about to overwrite still holds unclaimed ranges (its group's
// predecessors are late); wave 0 then resolves in the foreground.  No spill round trip (round 3's map + placement newline form moved every
// delimiter through HBM twice more), no coordinator wave and no placement launch (the one-pass look-back
// kernel's start and tail).  Deadlock-free: a workgroup publishes the AGG of every group it has scanned before
// it blocks, groups are claimed in increasing order by running workgroups, and a group's prefix depends only
// on lower groups, so the lowest unresolved group can always resolve.
// Shipped policies (each against its measured alternatives): 4 slots of 640 positions per range (5-8
// slots +-0.5 %; a 448 cap turned CSV ranges dense), placement shared by the first waves to arrive, b[1]'s reload
// before the placements, the look-back window issued at the step's end by wave 0 alone and reduced mid-next step, one
// group per claim, two-part windows.
constexpr uint32_t kLineSlots = 4;                 // steps of positions a workgroup holds in LDS
constexpr uint32_t kLineCap = 640;                 // positions kept per range; more = dense (rescanned)
static_assert(kLineSlots >= 3 && kLineSlots <= 8, "line slots: phase A, resolution, placement + slack");
static_assert(kLineCap % 8 == 0 && kLineCap <= 1024, "line cap");
constexpr uint32_t kLineGrpQ = 16;                 // claimed groups by step (>= slots + claim-ahead + 1)
static_assert(kLineGrpQ >= kLineSlots + kMapAhead + 1, "group queue spans the pending and claimed steps");
constexpr uint32_t kLineDense = 0x80000000u;
constexpr uint32_t kLineValid = 16u, kLineFirst = 32u, kLineLast = 64u;   // geo.z flag bits (lo_w < 16)
constexpr uint32_t kLineEnd = 128u;                // geo.z: the launch's last range (writes the total)
// A look-back window (kLineSpan descriptors before a group) arrives by LDS-DMA: kLineWinLoads 16-byte-per-lane
// loads from an even descriptor index, so 128 descriptors per load cover any kLineSpan before the group.
// Two parts: the nearest kLbSlots groups (~one round of the grid's claims) are reduced first; when all of them are
// published and none is resolved, the kLbSlots before them.  So a group's prefix does not wait for the round before
// it to be resolved, only for its AGGs (published without any dependency): a look-back limited to the round before
// chained every round's resolution to the last one's, and one late workgroup delayed all later ones.
constexpr uint32_t kLineSpan = kLbSlots * 2;
constexpr uint32_t kLineWinLoads = (kLineSpan + 2 + 2 * kWave - 1) / (2 * kWave);
constexpr uint32_t kLineWin = kLineWinLoads * kWave * 2;
static_assert(kLineWin >= kLineSpan + 2, "window loads cover kLineSpan descriptors from an even start");
// lb_window_dma clamps a window to the descriptor array's end: ensure_desc allocates multiples of 1024 descriptors
static_assert(kLineWin <= 1024, "a look-back window fits in the smallest descriptor array");
constexpr int kWinN = (int)kLineWinLoads;          // wave 0's window loads per step (no other wave issues any)

struct LineShared {
  uint16_t ev[kLineSlots][kMapWaves][kLineCap];    // per slot and wave: the range's positions
  uint4 geo[kLineSlots][kMapWaves];                // {wbase lo, wbase hi, lo_w | flags | hi_w << 16, chunk}
  uint32_t cnt[kLineSlots][kMapWaves];             // the range's delimiters (| kLineDense)
  uint32_t ex[kLineSlots][kMapWaves];              // delimiters of the group before the range (wave 0)
  unsigned long long pw[kLineSlots][kMapWaves];    // the range's launch prefix, valid once res == group + 1
  unsigned long long tot[kLineSlots];              // the group's delimiters
  uint32_t res[kLineSlots];
  uint32_t pclaim[kLineSlots];                     // ranges of the slot's step claimed for placement
  uint32_t grp[kLineGrpQ];                         // the group of step k at [k % kLineGrpQ]
  unsigned long long win[kLineWin];                // wave 0: a look-back window's descriptors, by LDS-DMA
  unsigned long long win_dummy[kLineWin];          // a step's window loads with no group to resolve (never read)
};

struct LineArgs {
  const uint8_t* base;          // = ScanArgs::base
  uint64_t nchunks, nranges;
  uint64_t desc_cap;            // descriptors allocated (a window load never reads past them)
  unsigned int* ticket;         // [2] group tickets: this launch claims from ticket[parity] and zeroes the other
  uint32_t parity;
  const uint32_t* pick;         // (auto form) the form dp_delim's density probe chose; run only when it is kFormLine
};

#ifdef DP_DIAG
#define LTL(step, e) do { const int lw_ = wave == 0 ? 0 : wave == 1 ? 1 : wave == 8 ? 2 : wave == 15 ? 3 : -1; \
    if (lw_ >= 0 && lane == 0 && blockIdx.x < 256 && (uint32_t)(step) < kLtlSteps) \
      g_prof[kLtlBase + (((uint64_t)blockIdx.x * kLtlSteps + (uint32_t)(step)) * kLtlWaves + lw_) * 8 + (e)] = \
          __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define LTL(step, e) do {} while (0)
#endif
// s_waitcnt vmcnt with the count of wave 0 (first) or of every other wave
template <int A0, int B0>
__device__ __forceinline__ void vm_wait2(bool first) {
  if (A0 == B0 || first) asm volatile("s_waitcnt vmcnt(%0)" :: "i"(A0) : "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" :: "i"(B0) : "memory");
}

// LDS byte address of a __shared__ object (the LDS-DMA destination base, M0)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// Look-back window of group u into LDS by LDS-DMA, hand-waited (inline asm: the compiler adds no wait, and no
// VGPR is held while the loads travel): descriptors [base, base + kLineWin) of which [u - kLineSpan, u) matter.
// Relaxed agent-scope reads (sc1), as ld_desc.  Returns base.
__device__ __forceinline__ uint64_t lb_window_dma(const ScanArgs& A, uint64_t desc_cap, uint32_t u, unsigned long long* win,
                                                  int lane) {
  uint64_t base = u > kLineSpan ? ((uint64_t)(u - kLineSpan) & ~1ull) : 0ull;
  if (base + kLineWin > desc_cap) base = desc_cap - kLineWin;      // (desc_cap: a multiple of 1024 >= kLineWin)
  const uint32_t dst = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_addr(win));
#pragma unroll
  for (uint32_t i = 0; i < kLineWinLoads; ++i) {
    const void* g = A.desc + base + i * 2u * kWave + 2u * (uint32_t)lane;
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(dst + i * 16u * kWave) : "memory");
  }
  return base;
}
// The window of group u from LDS, as lb_load lays it out.  Only after a wait that retired its LDS-DMA loads: the
// reads are tagged (`; dp_win_read`) and the ISA guard fails any such read that an LDS-DMA load may still be in
// flight at (isa_guard.py), so a reordered step cannot read another group's or a partial window.
__device__ __forceinline__ void lb_window_read(const unsigned long long* win, uint64_t base, uint32_t u, int lane,
                                               uint64_t (&d)[kLbPer]) {
  const uint32_t W = u < kLbSlots ? u : kLbSlots;
  const uint32_t rl = (uint32_t)(kWave - 1 - lane);
#pragma unroll
  for (int j = 0; j < kLbPer; ++j) {
    const uint32_t k = kLbPer * rl + j;
    const uint32_t idx = k < W ? (uint32_t)((uint64_t)(u - 1 - k) - base) : 0u;
    uint64_t v;
    asm volatile("ds_read_b64 %0, %1 ; dp_win_read\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(win + idx)) : "memory");
    d[j] = k < W ? v : 0ull;
  }
}
// Reduce a loaded window of group u: true with the group's launch prefix P once resolvable.
__device__ __forceinline__ bool lb_count_window(const ScanArgs& A, uint32_t u, uint64_t (&d)[kLbPer], int lane, uint64_t& P,
                                                bool* all = nullptr) {
  const uint32_t W = u < kLbSlots ? u : kLbSlots;
  const uint32_t rl = (uint32_t)(kWave - 1 - lane);
#pragma unroll
  for (int j = 0; j < kLbPer; ++j) {
    const uint32_t k = kLbPer * rl + j;
    d[j] = k < W ? ((d[j] & kEpochMask) == A.epoch ? d[j] : 0ull) : kIdentDesc;
  }
  return lb_reduce_count(d, W, pack_count(kStatPrefix, 0ull), lane, P, all);
}

template <int OUT64>
__global__ void __launch_bounds__(kWave * kMapWaves, 4) line_kernel(LineArgs L, ScanArgs A,
                                                                 const uint64_t* __restrict__ tab_lo,
                                                                 const uint64_t* __restrict__ tab_hi,
                                                                 const uint64_t* __restrict__ tab_r0) {
  static_assert(kMapWaves == 16, "line_kernel: one workgroup of 16 waves per CU");
  constexpr int kLoadsX = kLoadsPerBufN;
  __shared__ __attribute__((aligned(16))) LineShared sh;
  const int lane = __lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Tab T{(cu64*)tab_lo, (cu64*)tab_hi, (cu64*)tab_r0};
  const uint32_t nranges = (uint32_t)L.nranges, nchunks = (uint32_t)L.nchunks;
  const uint32_t ngroups = (nranges + kMapWaves - 1) / kMapWaves;
  unsigned int* ticket = L.ticket + L.parity;
  if (blockIdx.x == 0 && threadIdx.x == 0) L.ticket[L.parity ^ 1u] = 0u;   // the next launch's ticket
  if (L.pick != nullptr && *(const cu32s*)(uintptr_t)L.pick != kFormLine) return;   // (uniform) the probe chose the other form
  uint32_t claimed = 2, pend = 0, claim_res = 0;
  // Every group is claimed from the ticket, the first two as well (one atomic), never assigned by blockIdx: a
  // group then only ever waits on lower groups that running workgroups hold, so a grid need not be resident
  // all at once (two processes' grids sharing a GPU: with static first groups each grid's running workgroups
  // waited on its own unstarted ones, which waited for the other grid's CUs).
  if (threadIdx.x == 0) {
    const uint32_t u0 = atomicAdd(ticket, 2u);
    sh.grp[0] = u0;
    sh.grp[1] = u0 + 1u;
  }
  if (threadIdx.x < kLineSlots) sh.res[threadIdx.x] = 0u;
  __syncthreads();
  if (sh.grp[0] >= ngroups) return;                  // (uniform) every group went to another workgroup
  const uint32_t key = A.delim ^ kSel12;
  uint32_t r = sh.grp[0] * kMapWaves + (uint32_t)wave;
  Cursor cur{0, 0, 0, 0, 0, 0};
  Geo g = range_geo(T, nchunks, nranges, r, cur);
  BufN b[kBufs];
#pragma unroll
  for (int h = 0; h < kBufs; ++h) load_bufx(b[h], A, g, lane, h);
  bool ovf = false;
  uint32_t nb = 0;                                   // (every wave) the next step to place
  // (wave 0) steps with a published AGG / a resolved prefix, the step of the look-back window in flight and its
  // first descriptor (in registers: kept in LDS they cost wave 0 ~10 dependent LDS round trips per step, and the
  // barrier made every wave wait for them: 956 vs 849 us per 4 GiB CSV)
  uint32_t agg_next = 0, res_next = 0, lb_step = 0xFFFFFFFFu;
  uint64_t win_base = 0;

  // phase B of range w of step q (its geometry, count and prefix read from the slot up front: one LDS round trip)
  auto place = [&](uint32_t q, uint32_t w) {
    const uint32_t s = q % kLineSlots;
    const uint4 gq = sh.geo[s][w];
    const uint32_t cw = sh.cnt[s][w];
    const uint64_t Pw = sh.pw[s][w];
    if (!(gq.z & kLineValid)) return;
    const uint32_t n = cw & ~kLineDense;
    const uint64_t wbase = (uint64_t)gq.x | ((uint64_t)gq.y << 32);
    const uint32_t lo_w = gq.z & 15u, hi_w = gq.z >> 16;
    const uint64_t off0 = A.obj_base - A.shift + wbase;
    if (lane == 0) {
      if (gq.z & kLineLast) A.chunk_end[gq.w] = Pw + n;
      if (gq.z & kLineEnd) A.total[0] = Pw + n;
      if constexpr (OUT64 >= 2) {
        // the entries before every 64 KiB boundary that starts a range of this chunk (phase_b)
        const uint64_t j = (off0 >> 16) - A.tab_j0;
        if ((off0 & 0xFFFFull) == 0 && lo_w == 0 && hi_w != 0 && off0 >= (A.tab_j0 << 16) && j < A.tab_n)
          A.blocktab[j] = Pw;
      }
    }
    if (cw & kLineDense) {
      dense_b<kDelim, OUT64>(A, wbase, lo_w | (hi_w << 16), Pw, 0u, lane);
      return;
    }
    const uint16_t* evw = sh.ev[s][w];
    auto ev = [&](uint32_t i) { return (uint32_t)evw[i]; };
    // (uint64 output without the paired stores: their registers would push this kernel past 128 VGPRs)
    ovf |= place_delims<OUT64, false>(A, ev, n, Pw, off0, lane);
    if constexpr (OUT64 == 3) place_subs(A, ev, n, Pw, off0, (int)lo_w, (int)hi_w, lane);
  };
  // (wave 0) step q's AGG: the group's count from its 16 ranges (lanes 0..15), with every range's exclusive prefix
  auto publish_agg = [&](uint32_t q) {
    const uint32_t s = q % kLineSlots;
    const uint32_t c = lane < (int)kMapWaves ? (sh.cnt[s][lane] & ~kLineDense) : 0u;
    uint32_t inc = c;
    inc += dpp32<kRowShr1, 0xF>(inc, 0u);
    inc += dpp32<kRowShr2, 0xF>(inc, 0u);
    inc += dpp32<kRowShr4, 0xF>(inc, 0u);
    inc += dpp32<kRowShr8, 0xF>(inc, 0u);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, kMapWaves - 1);
    if (lane < (int)kMapWaves) sh.ex[s][lane] = inc - c;
    if (lane == 0) {
      sh.tot[s] = total;
      st_desc(&A.desc[sh.grp[q % kLineGrpQ]], pack_count(kStatAgg, total) | A.epoch);
    }
    agg_next = q + 1;
  };
  // (wave 0) a resolved prefix P: every range's prefix in LDS, the slot's tag for the other waves, the PREFIX
  // descriptor for the other workgroups
  auto resolved = [&](uint32_t q, uint64_t P) {
    const uint32_t s = q % kLineSlots;
    const uint32_t u = sh.grp[q % kLineGrpQ];
    if (lane < (int)kMapWaves) sh.pw[s][lane] = P + sh.ex[s][lane];   // every range's launch prefix
    const uint64_t pref = pack_count(kStatPrefix, P + sh.tot[s]);
    cbar();
    if (lane == 0) {
      lds_st(&sh.res[s], u + 1u);
      st_desc(&A.desc[u], pref | A.epoch);
    }
    res_next = q + 1;
  };
  // (wave 0) resolve every step up to q in the foreground (compiler-waited look-back loads)
  auto resolve_upto = [&](uint32_t q) {
    if (lb_step != 0xFFFFFFFFu) {                    // a hand-waited look-back in flight: let it land
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lb_step = 0xFFFFFFFFu;
    }
    uint64_t t0 = 0;
    uint32_t spins = 0;
    while (res_next <= q) {
      const uint32_t u = sh.grp[res_next % kLineGrpQ];
      const uint32_t W = u < kLbSlots ? u : kLbSlots;
      uint64_t d[kLbPer];
      const uint32_t rl = (uint32_t)(kWave - 1 - lane);
#pragma unroll
      for (int j = 0; j < kLbPer; ++j) {
        const uint32_t k = kLbPer * rl + j;
        d[j] = ld_desc(&A.desc[k < W ? u - 1 - k : 0u]);
      }
      uint64_t P = 0;
      if (lb_count_window(A, u, d, lane, P)) {
        resolved(res_next, P);
        continue;
      }
      if (wait_expired(spins++, t0)) {               // give up: flag it and release the waiting waves
        if (lane == 0) atomicOr(A.err, kErrTimeout);
        resolved(res_next, 0ull);
        continue;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  };
  auto resolved_tag = [&](uint32_t q) { return lds_ld(&sh.res[q % kLineSlots]) == sh.grp[q % kLineGrpQ] + 1u; };
  // (every wave) block until step q's prefix is known (wave 0 resolves it in the foreground)
  auto wait_resolved = [&](uint32_t q) {
    if (wave == 0) {
      resolve_upto(q);
    } else {
      uint64_t t0 = 0;
      for (uint32_t spins = 0; !resolved_tag(q); ++spins) {
        if (wait_expired(spins, t0)) {
          if (lane == 0) atomicOr(A.err, kErrTimeout);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    cbar();
  };
  // claim and place ranges of the resolved steps nb .. lim - 1, in order, without blocking: a claim is one LDS add
  // on the slot's counter; a step whose 16 ranges are all claimed is left behind (nb + 1).  A wave places what it
  // claims before it reaches the next barrier, so a step whose ranges are all claimed before the barrier is placed
  // after it; the slot stall makes every wave see its next slot's old step all claimed, and the slot's counter is
  // reset after that barrier, so no claim ever reaches a reused slot.
  auto help = [&](uint32_t lim) {
    while (nb < lim) {
      const uint32_t s0 = nb % kLineSlots;
      if (!resolved_tag(nb)) break;
      cbar();
      uint32_t w = 0;
      if (lane == 0) w = lds_add(&sh.pclaim[s0], 1u);
      w = rfl(w);
      if (w >= kMapWaves) {
        ++nb;
        continue;
      }
      place(nb, w);
    }
  };
  // (every wave) place steps nb .. q, waiting for their prefixes, until all their ranges are claimed
  auto place_upto = [&](uint32_t q) {
    while (nb <= q) {
      wait_resolved(nb);
      help(q + 1u);
    }
  };

  // Vector-memory order per step (vmcnt counts in issue order):
  // [b1 reload, placement stores, wave 0's window loads of the last step] | barrier | wait b0 (b1, those stores
  // and the window may stay in flight: a conservative count when there were stores) | claim atomic, wave 0's
  // AGG store | rows(0) | b0 reload | wait b1 (only b0's reload in flight: the claim and the window have landed)
  // | window reduction (wave 0) | rows(1) | b1 reload | placements | window loads (wave 0).  So a window travels
  // for half a step and no wait covers a load just issued.
  // (wave 0) reduce the look-back window that has landed (lb_step: the step of its group)
  auto consume = [&]() {
    if (lb_step == 0xFFFFFFFFu) return;
    const uint32_t q = lb_step, u = sh.grp[q % kLineGrpQ];
    lb_step = 0xFFFFFFFFu;
    uint64_t d[kLbPer];
    lb_window_read(sh.win, win_base, u, lane, d);
    uint64_t P = 0;
    bool all = false;
    bool ok = lb_count_window(A, u, d, lane, P, &all);
    if (!ok && all) {                                 // (u >= kLbSlots) the part before: its prefix + this sum
      const uint64_t S1 = P;
      lb_window_read(sh.win, win_base, u - kLbSlots, lane, d);
      ok = lb_count_window(A, u - kLbSlots, d, lane, P);
      P += S1;
    }
    if (ok) resolved(q, P);
  };
  // Wave 0 issues the window's kLineWinLoads LDS-DMA loads once per step, so its waits have one count on every
  // path (a count per path inside one branch made the compiler merge b[1]'s registers through copies above the
  // wait; one count per wave role, in uniform branches, does not).  Only the window of wave 0's oldest unresolved
  // group with a published AGG is read; with no such group the loads are lane 0's 16 bytes each (the count is per
  // instruction, the bytes per active lane) into a dummy area that is never read.
  auto issue_window = [&]() {
    const bool want = wave == 0 && res_next < agg_next;
    const uint32_t u = want ? sh.grp[res_next % kLineGrpQ] : 0u;
    uint64_t base = 0;
    if (wave == 0 && (want || lane == 0)) base = lb_window_dma(A, L.desc_cap, u, want ? sh.win : sh.win_dummy, lane);
    if (want) {
      win_base = base;
      lb_step = res_next;
    }
  };
  static_assert(kBufs == 2, "line_kernel: two input buffers per range");
  issue_window();                                     // (a dummy: the first step's wait counts a window)
  uint32_t it = 0;
  for (;; ++it) {
    __syncthreads();
    LTL(it, 0);
    if (threadIdx.x == 0) sh.pclaim[it % kLineSlots] = 0u;   // its old step: placed (last stall)
    const uint32_t gnext = sh.grp[(it + 1) % kLineGrpQ];
    const uint32_t rn = gnext < ngroups ? gnext * kMapWaves + (uint32_t)wave : nranges;
    const bool do_claim = wave == 0 && claimed < it + 1u + kMapAhead && sh.grp[(claimed - 1) % kLineGrpQ] < ngroups;
    const Geo gn = range_geo(T, nchunks, nranges, rn, cur);
    const uint32_t slot = it % kLineSlots;
    uint32_t nev = 0;
    const int lo = (int)g.lo_u, hi = (int)g.hi_u;
    const bool interior = lo == 0 && hi > kWaveBytes;   // wave-uniform
    uint16_t* evw = sh.ev[slot][wave];
    auto keep = [&](uint32_t rk, uint32_t pos) { evw[rk < kLineCap - 1u ? rk : kLineCap - 1u] = (uint16_t)pos; };
    v4u x[kRows];
    auto rows = [&](int h) {
#pragma unroll
      for (int i = 0; i < kRows; ++i) x[i] = b[h].x[i];
      if (interior) delim_rows<true>(x, h, lo, hi, key, lane, nev, keep);
      else delim_rows<false>(x, h, lo, hi, key, lane, nev, keep);
    };
    // ---- buffer 0
    // the youngest operations in flight: b[1]'s loads and, for wave 0, the window issued after them
    vm_wait2<kLoadsX + kWinN, kLoadsX>(wave == 0);
    touch_bufx(b[0]);
    __builtin_amdgcn_sched_barrier(0);
    LTL(it, 1);
    if (do_claim) {
      claim_res = atomic_add_nowait(ticket, 1u);
      pend = 1u;
    }
    // every wave wrote step it - 1's summary before the barrier: its AGG goes out before anything blocks
    if (wave == 0 && it > 0) publish_agg(it - 1);
    LTL(it, 2);
    rows(0);
    load_bufx(b[0], A, gn, lane, 0);
    // ---- buffer 1
    LTL(it, 3);
    vm_wait2<kLoadsX, kLoadsX>(wave == 0);            // b[0]'s reload in flight: the window and the claim have landed
    touch_bufx(b[1]);
    __builtin_amdgcn_sched_barrier(0);
    if (wave == 0) consume();                         // issued at the end of the last step, before b[0]'s reload
    if (pend) {                                       // the wait above covered the claim: its value is back
      asm volatile("" : "+v"(claim_res) :: "memory");
      const uint32_t u = rfl(claim_res);
      if (lane == 0)
        for (uint32_t i = 0; i < pend; ++i) sh.grp[(claimed + i) % kLineGrpQ] = u + i;
      claimed += pend;
      pend = 0;
    }
    LTL(it, 4);
    rows(1);
    cbar();
    if (lane == 0) {
      const bool valid = (g.fl & kGeoValid) != 0u;
      sh.cnt[slot][wave] = valid ? (nev | (nev > kLineCap ? kLineDense : 0u)) : 0u;
      sh.geo[slot][wave] = uint4{(uint32_t)g.ubase, (uint32_t)(g.ubase >> 32),
                                 g.lo_u | (valid ? kLineValid : 0u) | ((g.fl & kGeoFirst) ? kLineFirst : 0u) |
                                     ((g.fl & kGeoLast) ? kLineLast : 0u) | (r + 1u == nranges ? kLineEnd : 0u) |
                                     (g.hi_u << 16),
                                 g.c};
    }
    // this step's placements: any range of an older step whose prefix is known, claimed, so the waves that finish
    // their rows first place most of them; then, if the next step's slot still holds an unclaimed range, block for
    // it here (a claimed range is placed before its wave reaches the next barrier).  Blocking holds back this
    // workgroup's AGG of step it, its newest group, while it waits for an older one: the lowest waiting group
    // never depends on a held AGG.
    LTL(it, 5);
    load_bufx(b[kBufs - 1], A, gn, lane, kBufs - 1);
    help(it);
    LTL(it, 6);
    if (nb + kLineSlots <= it + 1) place_upto(it + 1 - kLineSlots);
    issue_window();
    LTL(it, 7);
    if (gnext >= ngroups) break;                      // uniform (LDS value read after the barrier)
    r = rn;
    g = gn;
  }
  drain_bufsx(b);                                     // (and a look-back window still in flight)
  if (wave == 0) lb_step = 0xFFFFFFFFu;
  __syncthreads();                                    // every wave's last summary is in LDS
  LTL(it + 1, 0);
  if (wave == 0) publish_agg(it);
  place_upto(it);
  LTL(it + 1, 1);
  if (ovf) atomicOr(A.err, kErrOverflow);
}

// x - pa clamped to 0..16 (the byte bound inside one 16-byte lane), without 32-bit truncation
__device__ __forceinline__ int lane_rel(uint64_t x, uint64_t pa) {
  return x <= pa ? 0 : (x - pa >= 16u ? 16 : (int)(x - pa));
}
// first position >= from (aligned coords) holding the delimiter, inside [from, end); -1 if none.  One wave.
__device__ uint64_t wave_find(const uint8_t* base, uint64_t from, uint64_t end, uint32_t pat, int lane, bool& found) {
  const uint32_t key = pat ^ kSel12;
  for (uint64_t a = from & ~15ull; a < end; a += kRowBytes) {
    const uint64_t pa = a + (uint64_t)lane * 16;
    uint32_t m = 0;
    // the lane's window [from, end) in its own 16 bytes, clamped in 64 bits: end - pa exceeds an int once the
    // buffer runs more than 2 GiB past `from` (a header cut by a chunk end early in a large buffer)
    if (pa < end) m = mask16(*reinterpret_cast<const uint4*>(base + pa), key) & range16(lane_rel(from, pa), lane_rel(end, pa));
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
    const uint64_t p = wave_find(R.base, R.chunk_hi[c], R.buf_end, 0x0A0A0A0Au, lane, found);
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
// Streaming ceilings on this device, reported next to the roofline fractions (tools/ubench_rw.hip has the
// variants these were chosen from): one 1024-thread workgroup per CU, each wave reading 16 KiB ranges as
// 16 non-temporal 16-byte lane loads in flight, and optionally writing `wq16 / 65536` output bytes per
// input byte as contiguous non-temporal 16-byte lane stores, range by range — the DELIM index's traffic
// mix (CSV ~0.22, VCF ~0.10).  Read-only: the best plain read rate measured (~7.0 TB/s on MI355X).
__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
  uint4 v;
  v.x = __builtin_nontemporal_load(&p->x);
  v.y = __builtin_nontemporal_load(&p->y);
  v.z = __builtin_nontemporal_load(&p->z);
  v.w = __builtin_nontemporal_load(&p->w);
  return v;
}
constexpr int kCalRange = 16384;
__global__ void __launch_bounds__(1024) stream_kernel(const uint4* __restrict__ in, uint64_t n16,
                                                     uint4* __restrict__ out, uint64_t wq16,
                                                     unsigned* __restrict__ sink) {
  const int lane = __lane_id();
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t nranges = (n16 * 16 + kCalRange - 1) / kCalRange;
  uint32_t acc = 0;
  for (uint64_t r = wave; r < nranges; r += nwaves) {
    const uint64_t i0 = r * (kCalRange / 16) + (uint64_t)lane;
    uint4 v[kCalRange / 1024];
#pragma unroll
    for (int i = 0; i < kCalRange / 1024; ++i) {
      const uint64_t j = i0 + (uint64_t)i * 64;
      v[i] = j < n16 ? ld_nt(in + j) : uint4{0u, 0u, 0u, 0u};
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < kCalRange / 1024; ++i) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    acc ^= x;
    if (out) {
      // one non-temporal 16-byte store per element (the scan's own output stores are 16-byte groups too)
      const uint64_t e0 = (r * wq16) >> 6, e1 = ((r + 1) * wq16) >> 6;   // 16-byte elements of this range
      for (uint64_t e = e0 + (uint64_t)lane; e < e1; e += 64)
        __builtin_nontemporal_store(v4u{x, (uint32_t)e, (uint32_t)r, acc}, reinterpret_cast<v4u*>(out) + e);
    }
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;   // keeps the loads alive; practically never stores
}

// The mixed read + write reference (round 3): the same reads, grouped as the scans group them — a workgroup
// step takes 16 consecutive 16 KiB ranges (one per wave), each wave's range in two 8 KiB halves whose next
// loads are issued before the step's stores — and the step's output as ONE contiguous run stored by all 1024
// threads after a workgroup barrier.  Of the shapes measured (tools/ubench_mix.hip, profiles/r03/
// ubench_mix*.log: per-range stores, compiler-pipelined, batched runs of 1 or 4 steps, stores one step late)
// this one moved the most bytes at the newline index's mixes: 3-9 % more than stream_kernel's per-range stores.
// (whole 16 KiB ranges only: a calibration tail below one range is not read)
__global__ void __launch_bounds__(1024) stream_rw_kernel(const uint4* __restrict__ in, uint64_t n16,
                                                        uint4* __restrict__ out, uint64_t wq16,
                                                        unsigned* __restrict__ sink) {
  constexpr int kHalfRows = kCalRange / 2048;          // 8 rows of 1 KiB per half
  __shared__ uint32_t s_x[16];
  const int lane = __lane_id();
  const int wave = (int)(threadIdx.x >> 6);
  const uint64_t nranges = n16 * 16 / kCalRange;
  const uint64_t ngroups = (nranges + 15) / 16;
  uint64_t grp = blockIdx.x;
  if (grp >= ngroups) return;
  uint32_t acc = 0;
  uint4 a[kHalfRows], b[kHalfRows];
  // a wave past the last range re-reads range 0 (its result is not stored)
  auto range_ptr = [&](uint64_t g) {
    const uint64_t r = g * 16 + (uint64_t)wave;
    return in + (r < nranges ? r : 0ull) * (kCalRange / 16) + lane;
  };
  const uint4* p = range_ptr(grp);
#pragma unroll
  for (int i = 0; i < kHalfRows; ++i) a[i] = ld_nt(p + i * 64);
#pragma unroll
  for (int i = 0; i < kHalfRows; ++i) b[i] = ld_nt(p + (kHalfRows + i) * 64);
  for (;;) {
    const uint64_t gn = grp + gridDim.x;
    const uint4* pn = range_ptr(gn < ngroups ? gn : grp);
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < kHalfRows; ++i) x ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
#pragma unroll
    for (int i = 0; i < kHalfRows; ++i) a[i] = ld_nt(pn + i * 64);
#pragma unroll
    for (int i = 0; i < kHalfRows; ++i) x ^= b[i].x ^ b[i].y ^ b[i].z ^ b[i].w;
#pragma unroll
    for (int i = 0; i < kHalfRows; ++i) b[i] = ld_nt(pn + (kHalfRows + i) * 64);
    acc ^= x;
    if (lane == 0) s_x[wave] = x;
    __syncthreads();
    // the group's run: elements [e(16 grp), e(16 grp + 16)) of e(r) = r * wq16 / 64
    const uint64_t r1 = grp * 16 + 16 < nranges ? grp * 16 + 16 : nranges;
    const uint64_t e0 = (grp * 16 * wq16) >> 6, e1 = (r1 * wq16) >> 6;
    const uint32_t xx = s_x[threadIdx.x & 15u];
    for (uint64_t e = e0 + threadIdx.x; e < e1; e += 1024)
      __builtin_nontemporal_store(v4u{xx, (uint32_t)e, (uint32_t)grp, acc}, reinterpret_cast<v4u*>(out) + e);
    __syncthreads();
    if (gn >= ngroups) break;
    grp = gn;
  }
#pragma unroll
  for (int i = 0; i < kHalfRows; ++i) acc ^= a[i].x ^ b[i].y;
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

// ------------------------------------------------------------------------------------------ newline form probe
// The newline kernels of a launch above kDelimLineMax bytes follow that launch's own bytes, chosen on the device (no
// host round trip): one workgroup reads kProbeSamples rows of 1 KiB spread evenly over the launch's ranges (their
// positions are part of the chunk table, stage_chunks) and counts their delimiters; at least dense_milli / 1000 per
// KiB picks line_kernel, fewer the one-pass look-back kernel.  Both are then enqueued and the one not picked returns
// at its first instruction.  A wave's 16 rows are loaded at once (one round trip, a few us per launch).
constexpr uint32_t kProbeSamples = 256;
constexpr uint32_t kProbeRowsPerWave = kProbeSamples / 16;
__global__ void __launch_bounds__(1024) density_probe_kernel(const uint8_t* base, uint32_t delim,
                                                             const uint64_t* __restrict__ samples, uint64_t dense_milli,
                                                             uint32_t* pick) {
  __shared__ uint32_t s_cnt, s_bytes;
  const int lane = __lane_id();
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t key = delim ^ kSel12;
  if (threadIdx.x == 0) {
    s_cnt = 0;
    s_bytes = 0;
  }
  __syncthreads();
  const cu64* smp = (const cu64*)samples;
  const int a = lane * 16;
  uint4 v[kProbeRowsPerWave];
  int lo[kProbeRowsPerWave], hi[kProbeRowsPerWave];
#pragma unroll
  for (uint32_t j = 0; j < kProbeRowsPerWave; ++j) {   // sample = {row start (aligned coordinate), lo | hi << 32}
    const uint32_t i = wave * kProbeRowsPerWave + j;
    const uint64_t row = smp[2 * i], w = smp[2 * i + 1];
    lo[j] = (int)(uint32_t)w;
    hi[j] = (int)(uint32_t)(w >> 32);
    // (the 16-byte block holding a range's last byte is read whole, as the scans' bounds-checked loads do)
    v[j] = (a < hi[j] && a + 16 > lo[j]) ? *reinterpret_cast<const uint4*>(base + row + (uint64_t)a) : uint4{0u, 0u, 0u, 0u};
  }
  uint32_t cnt = 0, bytes = 0;
#pragma unroll
  for (uint32_t j = 0; j < kProbeRowsPerWave; ++j) {
    cnt += (uint32_t)__popc(mask16(v[j], key) & range16(lo[j] - a, hi[j] - a));
    bytes += (uint32_t)(hi[j] - lo[j]);
  }
  atomicAdd(&s_cnt, cnt);
  if (lane == 0) atomicAdd(&s_bytes, bytes);
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t milli = s_bytes ? (uint64_t)s_cnt * 1024000ull / s_bytes : dense_milli;
    pick[0] = milli >= dense_milli ? kFormLine : kFormOne;
  }
}

// ------------------------------------------------------------------------------------------ host side
thread_local std::string g_err;

// Newline forms (profiles/r05/ sweeps, every form alternated rep by rep on one box): line_kernel is the
// faster form at every size for CSV-dense input (~28 newlines per KiB: 2-8 % ahead of the one-pass kernel from 2 to
// 64 GiB) and up to 4 GiB for sparser input (VCF, ~12.5 per KiB: 2 GiB 0.761 vs 0.735 of 8 TB/s, 4 GiB even);
// above 4 GiB the one-pass look-back kernel streams sparse input 2-4 % faster (its 16-unit ring and 4,096 positions
// per wave are slack that sparse input fills slowly, while line_kernel's 4 slots hold 4 steps at any density).  So
// the default ("auto") takes line_kernel up to kDelimLineMax bytes per launch, and above it lets the density probe
// pick from the launch's own bytes (kLineDenseMilli).
constexpr uint64_t kDelimLineMax = 4ull << 30;
constexpr uint64_t kLineDenseMilli = 20000;     // delimiters per KiB x 1000

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

// One scan stream per device, owned by the library.  Every scan launch of every context on a device goes
// to it, in call order: one grid fills the chip, so two scans side by side would only split the CUs, and
// a process then holds at most one scan stream per device (GPU_MAX_HW_QUEUES is 4 on the box; four or more
// context streams each launching scans and waiting on one another's events were seen to stall a scan for
// ~0.5 s).  A launch hands over with two events: the scan stream waits for the context
// stream's earlier work (table upload, input copies), the context stream waits for the scan (resolve
// kernel, read-back); the scan's HIP timing events sit on the scan stream around the kernels alone.
struct DeviceSerial {
  std::mutex m;
  hipStream_t scan = nullptr;         // created on the device's first scan, kept for the process
};
constexpr int kMaxDevices = 64;
DeviceSerial g_serial[kMaxDevices];

struct dp_ctx {
  int device = 0;
  hipStream_t own = nullptr, stream = nullptr;
  int cus = 0;
  int grid = 0;                       // persistent one-pass scan grid
  // device workspace
  unsigned long long* d_desc = nullptr;
  uint64_t desc_cap = 0;
  uint32_t desc_epoch = 0;            // last launch's descriptor epoch (0: the array needs zeroing first)
  uint64_t* d_tab = nullptr;          // chunk table + results + control words (stage_chunks)
  uint64_t tab_cap = 0;               // in u64 words
  uint64_t* h_tab = nullptr;          // pinned mirror
  uint64_t h_cap = 0;
  std::vector<uint64_t> last_tab;     // last uploaded table (skip identical re-uploads)
  // two-kernel FASTA workspace: range records and event spill slots (grow-only)
  uint4* d_rec = nullptr;
  uint16_t* d_spill = nullptr;
  uint64_t rec_cap = 0;               // ranges
  // forms (dp_ctx_set_form): the defaults are the shipped choices; the others are for tests and A/B runs
  int fasta_form = 0;                 // DP_FORM_FASTA: 0 map + placement kernels, 1 the one-pass look-back kernel
  int delim_form = 0;                 // DP_FORM_DELIM: 0 auto, 1 line_kernel, 3 one-pass
  uint64_t delim_line_max = kDelimLineMax;      // DP_FORM_DELIM_LINE_MAX
  uint64_t delim_dense_milli = kLineDenseMilli;  // DP_FORM_DELIM_DENSE
  uint32_t line_launches = 0;         // line_kernel launches (ticket parity)
  int delim_launched = 0;             // the newline launch in flight: its form, or 0 (picked on the device)
  int last_delim_form = 0;            // the kernels the last collected newline launch ran (1 or 3)
  // async call state
  int inflight = -1;                  // -1 none, kFasta, kDelim
  bool ctrl_pending = false;          // the launch's control words are already queued for read-back (enqueue_ctrl)
  uint64_t nchunks = 0, cap = 0;
  int out_u64 = 0;
  uint32_t every_k = 1;
  uint64_t carry = 0;
  std::vector<uint64_t> range_map;    // out_mode 3: caller range of each internal range (split at 64 KiB)
  uint64_t pend_off = 0, ctrl_off = 0, u0_off = 0;
  int last_form = -1;                 // the last scan's form on this ctx: 0 one-pass / line, 1 two kernels
  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  hipEvent_t ev_order = nullptr;      // dp_ctx_wait: device-scope ordering event on this ctx's stream
  hipEvent_t ev_in = nullptr;         // ctx stream -> device scan stream hand-over (DeviceSerial)
  hipEvent_t ev_out = nullptr;        // device scan stream -> ctx stream
  size_t ev_used = 0;
  double ms_acc = 0.0;
  uint64_t launches = 0;
};

std::atomic<uint64_t> g_dev_allocs{0}, g_host_allocs{0};

// The newline kernels of a launch scanning `span` bytes into `out_mode`: 1 line_kernel, 3 one-pass, or 0 when the
// launch's own bytes decide on the device (auto above delim_line_max).  The uint8 index (out_mode 4) takes line_kernel
// at every size: the one-pass kernel's phase B, on its data waves' path, pays for the 256-byte counts (VCF 16 GiB
// 2,740 vs line_kernel's 2,639 us, profiles/r05/u8).
static int delim_form_for(const dp_ctx* c, uint64_t span, int out_mode) {
  if (c->delim_form == (int)kFormLine || c->delim_form == (int)kFormOne) return c->delim_form;
  return span <= c->delim_line_max || out_mode == 4 ? (int)kFormLine : 0;
}

namespace {

// Every device / pinned host allocation the library makes goes through these (dp_alloc_counts).
hipError_t dev_alloc(void** p, uint64_t bytes) {
  g_dev_allocs.fetch_add(1, std::memory_order_relaxed);
  return hipMalloc(p, bytes);
}
hipError_t host_alloc(void** p, uint64_t bytes) {
  g_host_allocs.fetch_add(1, std::memory_order_relaxed);
  return hipHostMalloc(p, bytes, hipHostMallocDefault);
}

int ensure_tab(dp_ctx* c, uint64_t words) {
  if (words > c->tab_cap) {
    if (c->d_tab) HIPCHK(hipFree(c->d_tab));
    uint64_t cap = words + words / 2 + 64;
    HIPCHK(dev_alloc((void**)&c->d_tab, cap * 8));
    c->tab_cap = cap;
    c->last_tab.clear();   // forces a full upload (table + control words) before the next scan
  }
  if (words > c->h_cap) {
    if (c->h_tab) HIPCHK(hipHostFree(c->h_tab));
    uint64_t cap = words + words / 2 + 64;
    HIPCHK(host_alloc((void**)&c->h_tab, cap * 8));
    c->h_cap = cap;
  }
  return DP_OK;
}
// Look-back descriptors for a launch of `n` units / blocks / groups, and the launch's epoch tag (the array is zeroed
// only when (re)allocated and once every kEpochMax launches).  Multiples of 1024 (line_kernel's windows rely on it).
int next_epoch(dp_ctx* c, uint64_t n, uint64_t* epoch) {
  if (n > c->desc_cap) {
    if (c->d_desc) HIPCHK(hipFree(c->d_desc));
    c->d_desc = nullptr;
    c->desc_cap = 0;
    const uint64_t cap = ((n + n / 4 + 1023) / 1024) * 1024;
    HIPCHK(dev_alloc((void**)&c->d_desc, cap * 8));
    c->desc_cap = cap;
    c->desc_epoch = 0;
  }
  if (c->desc_epoch == 0 || c->desc_epoch >= kEpochMax) {   // fresh array, or the epochs wrapped
    HIPCHK(hipMemsetAsync(c->d_desc, 0, c->desc_cap * 8, c->stream));
    c->desc_epoch = 0;
  }
  *epoch = (uint64_t)(++c->desc_epoch) << kEpochShift;
  return DP_OK;
}
int ev_begin(dp_ctx* c, hipStream_t s) {
  if (!c->timing) return DP_OK;
  while (c->ev_pool.size() < c->ev_used + 2) {
    hipEvent_t e;
    // timing only (the result is collected after a stream sync): no system-scope fence, whose cache
    // writeback + invalidate at the record slows the bracketed scan by ~8% (measured, rocprofv3)
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    c->ev_pool.push_back(e);
  }
  HIPCHK(hipEventRecord(c->ev_pool[c->ev_used], s));
  return DP_OK;
}
int ev_end(dp_ctx* c, hipStream_t s) {
  if (!c->timing) return DP_OK;
  HIPCHK(hipEventRecord(c->ev_pool[c->ev_used + 1], s));
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

// Lay out the chunk table in aligned coordinates and enqueue its upload when it changed.
// Table layout (u64 words): lo[n] hi[n] r0[n+1] pending[n] chunk_end[n] ctrl[8] u0[n+1] probe[2 * kProbeSamples]:
// r0 = each chunk's first 16 KiB range (the two-kernel and lockstep kernels), u0 = its first 240 KiB unit (the one-pass
// kernel), probe = the density probe's sampled rows; ctrl =
// err | total | spare x2 (count-only scratch) | the one-pass unit ticket {next unit, workgroups finished} | the map
// kernel's group ticket (the same pair; zero between launches) | line_kernel's two group tickets (a launch claims
// from one half and zeroes the other, the next launch's) | the density probe's pick.
// No per-launch reset: every launch rewrites pending / chunk_end of each non-empty chunk and total (when it
// has units), so only the upload sets their defaults (-1, ~0, 0) and err = 0.  A launch that sets an err
// bit drops last_tab, so the next one re-uploads (results of a failed launch are discarded anyway).
constexpr uint64_t kCtrlWords = 8;
int stage_chunks(dp_ctx* c, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base, const uint64_t* chunks,
                 uint64_t n, uint64_t* nranges_out, uint64_t* nunits_out) {
  const uint64_t shift = (uint64_t)((uintptr_t)d_buf & 15u);
  const uint64_t words = 5 * n + 1 + kCtrlWords + n + 1 + 2 * kProbeSamples;
  std::vector<uint64_t> tab(3 * n + 1 + n + 1 + 2 * kProbeSamples);
  uint64_t ranges = 0, units = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t c0 = chunks[2 * i], c1 = chunks[2 * i + 1];
    if (c1 < c0 || c0 < buf_base || c1 > buf_base + buf_len)
      return fail(DP_ERR_INVALID, "chunk " + std::to_string(i) + " [" + std::to_string(c0) + "," +
                                      std::to_string(c1) + ") outside the buffer");
    const uint64_t lo = c0 - buf_base + shift, hi = c1 - buf_base + shift;
    tab[i] = lo;
    tab[n + i] = hi;
    tab[2 * n + i] = ranges;
    tab[3 * n + 1 + i] = units;
    if (hi > lo) {
      ranges += (hi - (lo & ~15ull) + kWaveBytes - 1) / kWaveBytes;
      units += (hi - (lo & ~15ull) + kUnitBytes - 1) / kUnitBytes;
    }
  }
  tab[3 * n] = ranges;
  tab[4 * n + 1] = units;
  // the density probe's rows: sample i at byte (2i + 1) * span / (2 kProbeSamples) of the chunks' bytes in order, its
  // 1 KiB row from the 16-byte block holding it, with the row's bytes inside the chunk as [lo, hi)
  uint64_t span = 0;
  for (uint64_t i = 0; i < n; ++i) span += tab[n + i] - tab[i];
  uint64_t* smp = tab.data() + 4 * n + 2;
  for (uint64_t i = 0, c = 0, before = 0; i < kProbeSamples && span; ++i) {
    const uint64_t p = ((2 * i + 1) * span) / (2 * kProbeSamples);
    while (before + (tab[n + c] - tab[c]) <= p) {
      before += tab[n + c] - tab[c];
      ++c;
    }
    const uint64_t pos = tab[c] + (p - before), row = pos & ~15ull;
    const uint64_t lo = tab[c] > row ? tab[c] - row : 0, hi = tab[n + c] - row < 1024 ? tab[n + c] - row : 1024;
    smp[2 * i] = row;
    smp[2 * i + 1] = lo | (hi << 32);
  }
  int rc = ensure_tab(c, words);
  if (rc) return rc;
  c->pend_off = 3 * n + 1;
  c->ctrl_off = 5 * n + 1;
  c->u0_off = c->ctrl_off + kCtrlWords;
  if (tab != c->last_tab) {
    // the pinned mirror may still feed an earlier async copy: wait for the stream before rewriting it
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(c->h_tab, tab.data(), (3 * n + 1) * 8);
    memset(c->h_tab + c->pend_off, 0xFF, 2 * n * 8);
    memset(c->h_tab + c->ctrl_off, 0, kCtrlWords * 8);
    memcpy(c->h_tab + c->u0_off, tab.data() + 3 * n + 1, (n + 1 + 2 * kProbeSamples) * 8);
    HIPCHK(hipMemcpyAsync(c->d_tab, c->h_tab, words * 8, hipMemcpyHostToDevice, c->stream));
    c->last_tab.swap(tab);
  }
  *nranges_out = ranges;
  *nunits_out = units;
  return DP_OK;
}

// Hand a scan over to the device's scan stream (caller holds ds.m): the scan stream waits for everything
// enqueued on the ctx stream so far.  scan_leave: the ctx stream waits for the scan.  Both events keep the
// default system-scope release: the input arrives by DMA and the read-back leaves by DMA.
int scan_enter(dp_ctx* c, DeviceSerial& ds, hipStream_t* ss) {
  if (!ds.scan) HIPCHK(hipStreamCreateWithFlags(&ds.scan, hipStreamNonBlocking));
  if (!c->ev_in) HIPCHK(hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming));
  if (!c->ev_out) HIPCHK(hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming));
  HIPCHK(hipEventRecord(c->ev_in, c->stream));
  HIPCHK(hipStreamWaitEvent(ds.scan, c->ev_in, 0));
  *ss = ds.scan;
  return DP_OK;
}
int scan_leave(dp_ctx* c, hipStream_t ss) {
  HIPCHK(hipEventRecord(c->ev_out, ss));
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_out, 0));
  return DP_OK;
}
// One scan on the device's scan stream: the hand-over, the timing events around the kernels `enq` enqueues on it
// (one HIP-event span per launch, however many kernels), the hand-back.  The device's lock is held throughout.
template <class Enq>
int on_scan_stream(dp_ctx* c, Enq&& enq) {
  DeviceSerial& ds = g_serial[c->device];
  std::lock_guard<std::mutex> lock(ds.m);
  hipStream_t ss = nullptr;
  int rc = scan_enter(c, ds, &ss);
  if (rc) return rc;
  rc = ev_begin(c, ss);
  if (rc) return rc;
  rc = enq(ss);
  if (rc) return rc;
  rc = ev_end(c, ss);
  if (rc) return rc;
  return scan_leave(c, ss);
}

// The arguments every scan kernel shares (a count-only call stores into the ctrl scratch words); the epoch is set by
// the caller (next_epoch).
ScanArgs scan_args(dp_ctx* c, const uint8_t* d_buf, uint64_t buf_base, uint64_t n, uint64_t nunits, void* d_out,
                   int kind, uint64_t cap, uint32_t delim, uint32_t every_k, uint32_t emit_add, uint64_t carry,
                   uint32_t wrap32, unsigned long long* blocktab, uint64_t tab_j0, uint64_t tab_n) {
  const uint64_t shift = (uint64_t)((uintptr_t)d_buf & 15u);
  ScanArgs a;
  memset(&a, 0, sizeof(a));
  a.base = d_buf - shift;
  a.shift = shift;
  a.obj_base = buf_base;
  a.nchunks = n;
  a.nunits = nunits;
  a.desc = c->d_desc;
  if (cap == 0 || d_out == nullptr) {                 // count-only call: stores go to a scratch slot
    d_out = c->d_tab + c->ctrl_off + 2;                // ctrl spare words (16 B: one uint64 pair)
    cap = 1;
  }
  a.out = d_out;
  a.cap = cap;
  a.out_u64 = kind;
  a.wrap32 = wrap32;
  a.blocktab = blocktab;
  a.tab_j0 = tab_j0;
  a.tab_n = tab_n;
  a.carry = carry;
  a.delim = delim * 0x01010101u;
  a.every_k = every_k;
  a.emit_add = emit_add;
  a.err = reinterpret_cast<uint32_t*>(c->d_tab + c->ctrl_off);
  a.total = reinterpret_cast<unsigned long long*>(c->d_tab + c->ctrl_off + 1);
  a.ticket = reinterpret_cast<unsigned int*>(c->d_tab + c->ctrl_off + 4);
  a.pending = reinterpret_cast<long long*>(c->d_tab + c->pend_off);
  a.chunk_end = reinterpret_cast<unsigned long long*>(c->d_tab + c->pend_off + n);
  a.pick = nullptr;
  return a;
}

// ctrl[4] is the one-pass kernel's unit ticket {next unit, workgroups finished}, which its last workgroup puts back
// to zero; a two-kernel launch leaves its placement block ticket there ({nblocks, 0}, zeroed only by the next map
// kernel): zero it before a one-pass launch that follows one (on the ctx stream, ahead of the hand-over).
int before_onepass(dp_ctx* c) {
  if (c->last_form == 1) HIPCHK(hipMemsetAsync(c->d_tab + c->ctrl_off + 4, 0, 8, c->stream));
  c->last_form = 0;
  return DP_OK;
}

// The one-pass look-back kernel over the 240 KiB-unit table (a.pick: run only if the density probe picked it).
int enq_scan(dp_ctx* c, hipStream_t ss, int mode, int kind, const ScanArgs& a) {
  const uint64_t n = a.nchunks, units = a.nunits;
  const unsigned grid = (unsigned)(units < (uint64_t)c->grid ? units : (uint64_t)c->grid);
  const uint64_t* tlo = c->d_tab;
  const uint64_t* thi = c->d_tab + n;
  const uint64_t* tu0 = c->d_tab + c->u0_off;
  if (mode == kFasta && !kind)
    hipLaunchKernelGGL((scan_kernel<kFasta, 0>), dim3(grid), dim3(kThreads), 0, ss, a, tlo, thi, tu0);
  else if (mode == kFasta)
    hipLaunchKernelGGL((scan_kernel<kFasta, 1>), dim3(grid), dim3(kThreads), 0, ss, a, tlo, thi, tu0);
  else if (kind == 2)
    hipLaunchKernelGGL((scan_kernel<kDelim, 2>), dim3(grid), dim3(kThreads), 0, ss, a, tlo, thi, tu0);
  else if (kind == 3)
    hipLaunchKernelGGL((scan_kernel<kDelim, 3>), dim3(grid), dim3(kThreads), 0, ss, a, tlo, thi, tu0);
  else if (kind == 0)
    hipLaunchKernelGGL((scan_kernel<kDelim, 0>), dim3(grid), dim3(kThreads), 0, ss, a, tlo, thi, tu0);
  else
    hipLaunchKernelGGL((scan_kernel<kDelim, 1>), dim3(grid), dim3(kThreads), 0, ss, a, tlo, thi, tu0);
  HIPCHK(hipGetLastError());
  return DP_OK;
}

// Range records and spill slots for a two-kernel FASTA launch (grow-only).
int ensure_ranges(dp_ctx* c, uint64_t nranges) {
  if (nranges >= 0xFFFFFFFFull) return fail(DP_ERR_INVALID, "launch exceeds 2^32 ranges of 16 KiB");
  if (nranges > c->rec_cap) {
    if (c->d_rec) HIPCHK(hipFree(c->d_rec));
    if (c->d_spill) HIPCHK(hipFree(c->d_spill));
    c->d_rec = nullptr;
    c->d_spill = nullptr;
    c->rec_cap = 0;
    const uint64_t cap_r = nranges + nranges / 8 + 64;
    HIPCHK(dev_alloc((void**)&c->d_rec, cap_r * sizeof(uint4)));
    const hipError_t e = dev_alloc((void**)&c->d_spill, cap_r * kSpillCap * sizeof(uint16_t));
    if (e != hipSuccess) {                             // leave no half-allocated workspace behind
      (void)hipFree(c->d_rec);
      c->d_rec = nullptr;
      c->d_spill = nullptr;
      return fail(DP_ERR_HIP, std::string("workspace of ") + std::to_string(nranges) + " ranges: " +
                                  hipGetErrorString(e));
    }
    c->rec_cap = cap_r;
  }
  return DP_OK;
}

MapArgs map_args(dp_ctx* c, const ScanArgs& a, uint64_t nranges) {
  MapArgs m;
  m.base = a.base;
  m.nchunks = a.nchunks;
  m.nranges = nranges;
  m.rec = c->d_rec;
  m.spill = c->d_spill;
  m.ticket = reinterpret_cast<unsigned int*>(c->d_tab + c->ctrl_off + 5);
  m.place_ticket = a.ticket;
  return m;
}
unsigned map_grid(const dp_ctx* c, uint64_t nranges) {
  const uint64_t groups = (nranges + kMapWaves - 1) / kMapWaves;
  return (unsigned)(groups < (uint64_t)c->cus ? groups : (uint64_t)c->cus);
}

// The two-kernel FASTA index (map_kernel + fasta_place_kernel) over the 16 KiB-range table.
int enq_fasta2(dp_ctx* c, hipStream_t ss, int out_u64, const ScanArgs& a, uint64_t nranges, bool count_only) {
  const uint64_t n = a.nchunks;
  const uint64_t nblocks = (nranges + kPlaceBlock - 1) / kPlaceBlock;
  const MapArgs m = map_args(c, a, nranges);
  PlaceArgs pa;
  pa.map_ticket = m.ticket;
  pa.rec = c->d_rec;
  pa.spill = c->d_spill;
  pa.nranges = nranges;
  pa.nblocks = nblocks;
  pa.count_only = count_only;
  pa.in_order = nblocks <= kLbSlots;                 // every window then reaches the base (b < kLbSlots)
  const uint64_t* tlo = c->d_tab;
  const uint64_t* thi = c->d_tab + n;
  const uint64_t* tr0 = c->d_tab + 2 * n;
  hipLaunchKernelGGL(map_kernel, dim3(map_grid(c, nranges)), dim3(kWave * kMapWaves), 0, ss, m, tlo, thi, tr0);
  HIPCHK(hipGetLastError());
  if (out_u64)
    hipLaunchKernelGGL((fasta_place_kernel<1>), dim3((unsigned)nblocks), dim3(kPlaceBlock), 0, ss, pa, a, tlo, thi, tr0);
  else
    hipLaunchKernelGGL((fasta_place_kernel<0>), dim3((unsigned)nblocks), dim3(kPlaceBlock), 0, ss, pa, a, tlo, thi, tr0);
  HIPCHK(hipGetLastError());
  return DP_OK;
}

// The lockstep newline kernel (line_kernel) over the 16 KiB-range table (pick: run only if the probe picked it).  The
// ticket parity advances only once the launch is enqueued: a launch that never ran must not leave the next one
// claiming from a ticket nobody zeroed.
int enq_line(dp_ctx* c, hipStream_t ss, int kind, const ScanArgs& a, uint64_t nranges, const uint32_t* pick) {
  const uint64_t n = a.nchunks;
  LineArgs L;
  L.base = a.base;
  L.nchunks = n;
  L.nranges = nranges;
  L.desc_cap = c->desc_cap;
  L.ticket = reinterpret_cast<unsigned int*>(c->d_tab + c->ctrl_off + 6);
  L.parity = c->line_launches & 1u;
  L.pick = pick;
  const uint64_t* tlo = c->d_tab;
  const uint64_t* thi = c->d_tab + n;
  const uint64_t* tr0 = c->d_tab + 2 * n;
  const dim3 grid(map_grid(c, nranges)), blk(kWave * kMapWaves);
  if (kind == 1) hipLaunchKernelGGL((line_kernel<1>), grid, blk, 0, ss, L, a, tlo, thi, tr0);
  else if (kind == 2) hipLaunchKernelGGL((line_kernel<2>), grid, blk, 0, ss, L, a, tlo, thi, tr0);
  else if (kind == 3) hipLaunchKernelGGL((line_kernel<3>), grid, blk, 0, ss, L, a, tlo, thi, tr0);
  else hipLaunchKernelGGL((line_kernel<0>), grid, blk, 0, ss, L, a, tlo, thi, tr0);
  HIPCHK(hipGetLastError());
  ++c->line_launches;
  return DP_OK;
}

// The density probe of an auto newline launch: its pick goes to ctrl[7].
int enq_probe(dp_ctx* c, hipStream_t ss, const ScanArgs& a, uint64_t nranges) {
  const uint64_t n = a.nchunks;
  (void)n;
  (void)nranges;
  hipLaunchKernelGGL(density_probe_kernel, dim3(1), dim3(1024), 0, ss, a.base, a.delim, c->d_tab + c->u0_off + n + 1,
                     c->delim_dense_milli, reinterpret_cast<uint32_t*>(c->d_tab + c->ctrl_off + 7));
  HIPCHK(hipGetLastError());
  return DP_OK;
}

int check_ctx(dp_ctx* c) {
  if (!c) return fail(DP_ERR_INVALID, "null dp_ctx");
  HIPCHK(hipSetDevice(c->device));
  return DP_OK;
}

// D2H of [pending (nchunks) | chunk_end (nchunks) | ctrl], queued on the context stream right behind a launch's
// kernels: a read-back queued only when the result is collected waits in the copy engine behind whatever other
// streams queued meanwhile (a streamed index's next H2D pieces: tens of ms).
int enqueue_ctrl(dp_ctx* c) {
  const uint64_t off = c->pend_off;
  const uint64_t words = c->ctrl_off + kCtrlWords - off;
  HIPCHK(hipMemcpyAsync(c->h_tab + off, c->d_tab + off, words * 8, hipMemcpyDeviceToHost, c->stream));
  c->ctrl_pending = true;
  return DP_OK;
}

int collect_ctrl(dp_ctx* c) {
  // the control words (queued at launch) and wait
  if (!c->ctrl_pending) {
    const int rc = enqueue_ctrl(c);
    if (rc) return rc;
  }
  c->ctrl_pending = false;
  HIPCHK(hipStreamSynchronize(c->stream));
  int rc = harvest_events(c);
  if (rc) return rc;
  return DP_OK;
}

}  // namespace

extern "C" {

int dp_abi_version(void) { return DP_ABI_VERSION; }

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
  if (device < 0 || device >= n || device >= kMaxDevices)
    return fail(DP_ERR_INVALID, "device " + std::to_string(device) + " out of range");
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
                          (const void*)scan_kernel<kDelim, 1>, (const void*)scan_kernel<kDelim, 2>,
                          (const void*)scan_kernel<kDelim, 3>};
  for (const void* k : others) {
    int o = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k, kThreads, 0));
    if (o < occ) occ = o;
  }
  // every workgroup of the one-pass kernel's persistent grid must be resident (look-back waits on lower units):
  // one 1024-thread workgroup per CU (the occupancy answer can over-report by one, MI355X_MICROARCH.md
  // §Residency), and G <= 256 keeps a unit's look-back one window
  if (occ < 1) {
    delete c;
    return fail(DP_ERR_HIP, "scan_kernel: no resident workgroup per CU");
  }
  c->grid = c->cus < 256 ? c->cus : 256;
  *out = c;
  return DP_OK;
}

int dp_ctx_destroy(dp_ctx* c) {
  if (!c) return DP_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto e : c->ev_pool) (void)hipEventDestroy(e);
  if (c->ev_order) (void)hipEventDestroy(c->ev_order);
  if (c->ev_in) (void)hipEventDestroy(c->ev_in);
  if (c->ev_out) (void)hipEventDestroy(c->ev_out);
  if (c->d_desc) (void)hipFree(c->d_desc);
  if (c->d_rec) (void)hipFree(c->d_rec);
  if (c->d_spill) (void)hipFree(c->d_spill);
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

int dp_ctx_wait(dp_ctx* c, dp_ctx* other) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (!other) return fail(DP_ERR_INVALID, "null other ctx");
  if (other->device != c->device) return fail(DP_ERR_INVALID, "contexts on different devices");
  if (!other->ev_order)
    HIPCHK(hipEventCreateWithFlags(&other->ev_order, hipEventDisableTiming | hipEventReleaseToDevice));
  HIPCHK(hipEventRecord(other->ev_order, other->stream));
  HIPCHK(hipStreamWaitEvent(c->stream, other->ev_order, 0));
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
  HIPCHK(dev_alloc(p, bytes ? bytes : 16));
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
  HIPCHK(host_alloc(p, bytes ? bytes : 16));
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
  uint64_t nranges = 0, units = 0;
  rc = stage_chunks(c, d_buf, buf_len, buf_base, chunks, nchunks, &nranges, &units);
  if (rc) return rc;
  const bool count_only = cap_pairs == 0 || d_out == nullptr;
  if (c->fasta_form == 1 && units) {                  // the one-pass look-back kernel (A/B)
    rc = before_onepass(c);
    if (rc) return rc;
    ScanArgs a = scan_args(c, d_buf, buf_base, nchunks, units, d_out, out_u64, cap_pairs, 0, 1, 0, 0, 0, nullptr, 0, 0);
    rc = next_epoch(c, units, &a.epoch);
    if (rc) return rc;
    a.desc = c->d_desc;
    rc = on_scan_stream(c, [&](hipStream_t ss) { return enq_scan(c, ss, kFasta, out_u64, a); });
  } else if (nranges) {                               // map_kernel + fasta_place_kernel
    rc = ensure_ranges(c, nranges);
    if (rc) return rc;
    ScanArgs a = scan_args(c, d_buf, buf_base, nchunks, nranges, d_out, out_u64, cap_pairs, 0, 1, 0, 0, 0, nullptr, 0, 0);
    rc = next_epoch(c, (nranges + kPlaceBlock - 1) / kPlaceBlock, &a.epoch);
    if (rc) return rc;
    a.desc = c->d_desc;
    c->last_form = 1;
    rc = on_scan_stream(c, [&](hipStream_t ss) { return enq_fasta2(c, ss, out_u64, a, nranges, count_only); });
  }
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
  return enqueue_ctrl(c);
}

int dp_fasta_result(dp_ctx* c, uint64_t* n_pairs, int64_t* pending, uint64_t* chunk_end) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (c->inflight != kFasta) return fail(DP_ERR_INVALID, "no FASTA scan in flight on this ctx");
  c->inflight = -1;
  rc = collect_ctrl(c);
  if (rc) return rc;
  const uint32_t err = (uint32_t)c->h_tab[c->ctrl_off];
  if (err) c->last_tab.clear();                         // the next launch re-uploads err = 0
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
  if (err & kErrTimeout) return fail(DP_ERR_TIMEOUT, "look-back wait timed out");
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

int dp_delim_ranges_async(dp_ctx* c, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base, const uint64_t* ranges,
                          uint64_t nranges, uint32_t delim, uint32_t every_k, uint32_t emit_add, uint64_t carry,
                          void* d_out, int out_mode, uint64_t cap) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (c->inflight >= 0) return fail(DP_ERR_INVALID, "a scan is already in flight on this ctx");
  if (every_k == 0) return fail(DP_ERR_INVALID, "every_k must be >= 1");
  if (delim > 255) return fail(DP_ERR_INVALID, "delim must be a byte");
  if (out_mode < 0 || out_mode > 4)
    return fail(DP_ERR_INVALID, "out_mode must be 0 (uint32), 1 (uint64), 2 (uint32 low words), 3 (uint16 + blocks) or "
                                "4 (uint8 + 256-byte counts + blocks)");
  if (nranges == 0 || !ranges) return fail(DP_ERR_INVALID, "no ranges");
  const bool blocked = out_mode >= 3;
  const std::string om = "out_mode " + std::to_string(out_mode);
  // the block tables hold delimiter ordinals before each 64 KiB / 256-byte boundary: entry indexes only when every
  // delimiter is an entry, and the low 16 / 8 bits locate an entry in its block only without an added offset
  if (blocked && (every_k != 1 || emit_add != 0))
    return fail(DP_ERR_INVALID, om + " needs every_k == 1 and emit_add == 0");
  for (uint64_t i = 0; i < nranges; ++i) {
    if (ranges[2 * i + 1] > ranges[2 * i] && !d_buf) return fail(DP_ERR_INVALID, "null buffer");
    if (ranges[2 * i + 1] < ranges[2 * i]) return fail(DP_ERR_INVALID, "range end before its start");
    if (i && ranges[2 * i] < ranges[2 * i - 1]) return fail(DP_ERR_INVALID, "ranges must ascend without overlap");
    if (blocked && i && ranges[2 * i] != ranges[2 * i - 1])
      return fail(DP_ERR_INVALID, om + " needs contiguous ranges");
  }
  if (cap && !d_out) return fail(DP_ERR_INVALID, "null output with cap > 0");
  // out_mode 3 / 4: split each range at its first 64 KiB boundary, so that every later boundary starts a wave
  // range (the kernel records the entries before it there); the block table follows the entries in d_out, and for
  // out_mode 4 the 256-byte table follows the block table
  std::vector<uint64_t> rg(ranges, ranges + 2 * nranges);
  c->range_map.clear();
  unsigned long long* tab = nullptr;
  uint16_t* sub = nullptr;
  uint64_t j0 = 0, ntab = 0, s0 = 0, nsub = 0;
  if (blocked) {
    rg.clear();
    for (uint64_t i = 0; i < nranges; ++i) {
      const uint64_t lo = ranges[2 * i], hi = ranges[2 * i + 1];
      const uint64_t a64 = (lo + 0xFFFFull) & ~0xFFFFull;
      if (lo < a64 && a64 < hi) {
        rg.push_back(lo); rg.push_back(a64); c->range_map.push_back(i);
        rg.push_back(a64); rg.push_back(hi); c->range_map.push_back(i);
      } else {
        rg.push_back(lo); rg.push_back(hi); c->range_map.push_back(i);
      }
    }
    // wave ranges start 16-byte aligned in buffer coordinates: object offsets must share that alignment
    if ((((uintptr_t)d_buf) - buf_base) & 15u)
      return fail(DP_ERR_INVALID, om + " needs d_buf and buf_base congruent mod 16 (place the bytes at "
                                       "an address whose low 4 bits equal buf_base's)");
    const uint64_t first = ranges[0], last = ranges[2 * nranges - 1];
    j0 = first >> 16;
    ntab = last > first ? ((last - 1) >> 16) - j0 + 1 : 1;
    const uint64_t item = out_mode == 3 ? 2 : 1;
    const uint64_t tab_off = (item * cap + 15) & ~15ull;
    tab = reinterpret_cast<unsigned long long*>(reinterpret_cast<uint8_t*>(d_out) + tab_off);
    if (out_mode == 4) {
      s0 = first >> 8;
      nsub = last > first ? ((last - 1) >> 8) - s0 + 1 : 1;
      sub = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(d_out) + ((tab_off + 8 * ntab + 15) & ~15ull));
    }
    if (!d_out) return fail(DP_ERR_INVALID, om + " needs an output buffer (entries + block tables)");
    if (((uintptr_t)d_out) & 15u) return fail(DP_ERR_INVALID, om + " needs a 16-byte aligned output buffer");
  }
  const uint64_t nr = rg.size() / 2;
  uint64_t nr16 = 0, units = 0, span = 0;
  for (uint64_t i = 0; i < nr; ++i) span += rg[2 * i + 1] - rg[2 * i];
  const int kind = out_mode == 1 ? 1 : out_mode == 3 ? 2 : out_mode == 4 ? 3 : 0;
  const int dform = delim_form_for(c, span, out_mode);
  rc = stage_chunks(c, d_buf, buf_len, buf_base, rg.data(), nr, &nr16, &units);
  if (rc) return rc;
  auto args = [&](uint64_t nu) {
    ScanArgs a = scan_args(c, d_buf, buf_base, nr, nu, d_out, kind, cap, delim, every_k, emit_add, carry, out_mode == 2,
                           tab, j0, ntab);
    a.subtab = sub;
    a.sub_s0 = s0;
    a.sub_n = nsub;
    return a;
  };
  const uint64_t ngroups = (nr16 + kMapWaves - 1) / kMapWaves;
  if (!nr16) {
    // nothing to scan (every range empty): no launch, the uploaded defaults are the result
  } else if (dform == (int)kFormLine) {               // the lockstep one-pass kernel
    ScanArgs a = args(nr16);
    rc = next_epoch(c, ngroups, &a.epoch);
    if (rc) return rc;
    a.desc = c->d_desc;
    c->last_form = 0;
    rc = on_scan_stream(c, [&](hipStream_t ss) { return enq_line(c, ss, kind, a, nr16, nullptr); });
  } else if (dform == (int)kFormOne) {                // the one-pass look-back kernel
    rc = before_onepass(c);
    if (rc) return rc;
    ScanArgs a = args(units);
    rc = next_epoch(c, units, &a.epoch);
    if (rc) return rc;
    a.desc = c->d_desc;
    rc = on_scan_stream(c, [&](hipStream_t ss) { return enq_scan(c, ss, kDelim, kind, a); });
  } else {                                            // auto: the density probe picks on the device
    rc = before_onepass(c);
    if (rc) return rc;
    ScanArgs a = args(units);
    rc = next_epoch(c, units > ngroups ? units : ngroups, &a.epoch);
    if (rc) return rc;
    a.desc = c->d_desc;
    const uint32_t* pick = reinterpret_cast<const uint32_t*>(c->d_tab + c->ctrl_off + 7);
    ScanArgs al = a, ao = a;
    al.nunits = nr16;
    ao.pick = pick;
    rc = on_scan_stream(c, [&](hipStream_t ss) {
      int r = enq_probe(c, ss, al, nr16);
      if (!r) r = enq_line(c, ss, kind, al, nr16, pick);
      if (!r) r = enq_scan(c, ss, kDelim, kind, ao);
      return r;
    });
  }
  if (rc) return rc;
  c->delim_launched = dform;
  c->inflight = kDelim;
  c->nchunks = nr;
  c->cap = cap;
  c->out_u64 = out_mode == 1;
  c->every_k = every_k;
  c->carry = carry;
  return enqueue_ctrl(c);
}

int dp_delim_ranges_result(dp_ctx* c, uint64_t* n_out, uint64_t* n_delims, uint64_t* range_end) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (c->inflight != kDelim) return fail(DP_ERR_INVALID, "no delimiter scan in flight on this ctx");
  const uint64_t k = c->every_k, carry = c->carry;
  c->inflight = -1;
  rc = collect_ctrl(c);
  if (rc) return rc;
  const uint32_t err = (uint32_t)c->h_tab[c->ctrl_off];
  if (err) c->last_tab.clear();                         // the next launch re-uploads err = 0
  // delimiters in the launch (the total is written at the last unit; no unit: none)
  uint64_t nd = 0;
  for (uint64_t i = 0; i < c->nchunks; ++i) {
    const uint64_t e = c->h_tab[c->pend_off + c->nchunks + i];
    if (e != ~0ull) nd = e;                             // empty ranges were never visited: carry the previous
    if (range_end) range_end[c->range_map.empty() ? i : c->range_map[i]] = nd;
  }
  const uint64_t nout = (carry + nd) / k - carry / k;
  c->last_delim_form = c->delim_launched ? c->delim_launched
                                          : (c->h_tab[c->ctrl_off + 7] == kFormLine ? (int)kFormLine : (int)kFormOne);
  if (n_delims) *n_delims = nd;
  if (n_out) *n_out = nout;
  if (err & kErrTimeout) return fail(DP_ERR_TIMEOUT, "look-back wait timed out");
  if (err & kErrOverflow) return fail(DP_ERR_OVERFLOW, "Python integer out of bounds for uint32");
  if (nout > c->cap) return fail(DP_ERR_CAPACITY, "output capacity " + std::to_string(c->cap) + " < " +
                                                      std::to_string(nout) + " offsets");
  return DP_OK;
}

int dp_delim_index_async(dp_ctx* c, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base, uint64_t begin,
                         uint64_t end, uint32_t delim, uint32_t every_k, uint32_t emit_add, void* d_out,
                         int out_u64, uint64_t cap) {
  const uint64_t r[2] = {begin, end};
  return dp_delim_ranges_async(c, d_buf, buf_len, buf_base, r, 1, delim, every_k, emit_add, 0, d_out, out_u64 ? 1 : 0,
                               cap);
}

int dp_delim_result(dp_ctx* c, uint64_t* n_out, uint64_t* n_delims) {
  return dp_delim_ranges_result(c, n_out, n_delims, nullptr);
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

int dp_stream_rw(dp_ctx* c, const void* d_in, uint64_t bytes, void* d_out, uint32_t write_q16, int blocks_per_cu) {
  int rc = check_ctx(c);
  if (rc) return rc;
  if (write_q16 && !d_out) return fail(DP_ERR_INVALID, "null output with write_q16 > 0");
  rc = ensure_tab(c, 8);
  if (rc) return rc;
  const int bpc = blocks_per_cu > 0 ? blocks_per_cu : 1;
  c->last_tab.clear();   // the table area is the (practically never written) sink
  // on the device's scan stream like a scan: a calibration never shares the chip with a scan of this process
  DeviceSerial& ds = g_serial[c->device];
  std::lock_guard<std::mutex> lock(ds.m);
  hipStream_t ss = nullptr;
  rc = scan_enter(c, ds, &ss);
  if (rc) return rc;
  rc = ev_begin(c, ss);
  if (rc) return rc;
  if (write_q16)
    hipLaunchKernelGGL(stream_rw_kernel, dim3((unsigned)(c->cus * bpc)), dim3(1024), 0, ss,
                       reinterpret_cast<const uint4*>(d_in), bytes / 16, reinterpret_cast<uint4*>(d_out),
                       (uint64_t)write_q16, reinterpret_cast<unsigned*>(c->d_tab));
  else
    hipLaunchKernelGGL(stream_kernel, dim3((unsigned)(c->cus * bpc)), dim3(1024), 0, ss,
                       reinterpret_cast<const uint4*>(d_in), bytes / 16, nullptr, 0ull,
                       reinterpret_cast<unsigned*>(c->d_tab));
  HIPCHK(hipGetLastError());
  rc = ev_end(c, ss);
  if (rc) return rc;
  return scan_leave(c, ss);
}

int dp_stream_read(dp_ctx* c, const void* d_buf, uint64_t bytes, int blocks_per_cu) {
  return dp_stream_rw(c, d_buf, bytes, nullptr, 0, blocks_per_cu);
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
#ifdef DP_DIAG
  if (!c || !host_words) return fail(DP_ERR_INVALID, "dp_debug_profile: null argument");
  const uint64_t n = n_words < kProfWords ? n_words : kProfWords;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpyFromSymbol(host_words, HIP_SYMBOL(g_prof), n * 8, 0, hipMemcpyDeviceToHost));
  if (slots) *slots = kProfSlots;
  if (waves) *waves = kProfWaves;
  return DP_OK;
#else
  (void)c; (void)host_words; (void)n_words; (void)slots; (void)waves;
  return fail(DP_ERR_INVALID, "dp_debug_profile: library built without -DDP_DIAG");
#endif
}

int dp_alloc_counts(uint64_t* device_allocs, uint64_t* host_allocs) {
  if (device_allocs) *device_allocs = g_dev_allocs.load(std::memory_order_relaxed);
  if (host_allocs) *host_allocs = g_host_allocs.load(std::memory_order_relaxed);
  return DP_OK;
}

int dp_ctx_set_form(dp_ctx* c, int what, uint64_t value) {
  if (!c) return fail(DP_ERR_INVALID, "null");
  if (c->inflight >= 0) return fail(DP_ERR_INVALID, "a scan is in flight on this ctx");
  switch (what) {
    case DP_FORM_FASTA:
      if (value > 1) return fail(DP_ERR_INVALID, "DP_FORM_FASTA: 0 (map + placement) or 1 (one-pass)");
      c->fasta_form = (int)value;
      return DP_OK;
    case DP_FORM_DELIM:
      if (value > 3 || value == 2) return fail(DP_ERR_INVALID, "DP_FORM_DELIM: 0 (auto), 1 (line_kernel) or 3 (one-pass)");
      c->delim_form = (int)value;
      return DP_OK;
    case DP_FORM_DELIM_LINE_MAX:
      c->delim_line_max = value;
      return DP_OK;
    case DP_FORM_DELIM_DENSE:
      c->delim_dense_milli = value;
      return DP_OK;
    default:
      return fail(DP_ERR_INVALID, "unknown form setting " + std::to_string(what));
  }
}

int dp_ctx_get_form(dp_ctx* c, int what, uint64_t* value) {
  if (!c || !value) return fail(DP_ERR_INVALID, "null");
  switch (what) {
    case DP_FORM_FASTA: *value = (uint64_t)c->fasta_form; return DP_OK;
    case DP_FORM_DELIM: *value = (uint64_t)c->delim_form; return DP_OK;
    case DP_FORM_DELIM_LINE_MAX: *value = c->delim_line_max; return DP_OK;
    case DP_FORM_DELIM_DENSE: *value = c->delim_dense_milli; return DP_OK;
    default: return fail(DP_ERR_INVALID, "unknown form setting " + std::to_string(what));
  }
}

int dp_last_delim_form(dp_ctx* c, int* form) {
  if (!c || !form) return fail(DP_ERR_INVALID, "null");
  *form = c->last_delim_form;
  return DP_OK;
}

int dp_scan_delim_form(dp_ctx* c, uint64_t span, int out_mode, int* form) {
  if (!c || !form) return fail(DP_ERR_INVALID, "null");
  *form = delim_form_for(c, span, out_mode);
  return DP_OK;
}

int dp_scan_geometry(dp_ctx* c, int* grid, int* unit_bytes) {
  if (!c) return fail(DP_ERR_INVALID, "null");
  if (grid) *grid = c->grid;
  if (unit_bytes) *unit_bytes = kUnitBytes;
  return DP_OK;
}

}  // extern "C"
