/*
 * dpscan.h — C ABI of libdpscan.so, the MI355X (gfx950) record-boundary scan behind dataplug_amd.
 *
 * Every entry point is a plain C function over raw pointers and sizes (no torch / HIP types in the
 * signatures; streams are opaque `void*` = hipStream_t).  Status is returned as an int (DP_OK = 0);
 * the message of the last failure on the calling thread is available from dp_last_error().  No C++
 * exception crosses this boundary.  A dp_ctx is bound to one device and owns one stream plus the
 * scan workspace; use one ctx per host thread (calls on distinct ctx are thread-safe, and ctypes
 * releases the GIL around them).  Scan kernels of every ctx on one device (in one process) run one after
 * another on one library-owned scan stream per device (one grid fills the chip); each scan call hands
 * over from the ctx stream to that stream and back with an event, so the ctx stream sees the results in
 * order.  Workgroups that depend on one another claim their work from a ticket at run time, so a grid
 * never waits on a workgroup that has not started: grids of different processes may share a GPU.
 *
 * Reference interfaces each entry point replaces (CLOUDLAB-URV/dataplug @ 2025-07-11):
 *   dp_fasta_index  <- dataplug/formats/genomics/fasta.py:24-63 (preprocess_fasta: the per-chunk
 *                      re.finditer(rb">.+(\n)?") scan at :36, the (start,end) pairs at :39-43, the
 *                      split-header end fix-up at :45-56 and the uint32 packing at :61-62), run for a
 *                      whole chunk plan at once (preprocessing/preprocess.py:38 + handler.py:36-38).
 *   dp_delim_index  <- the newline boundaries resolved byte-by-byte in CSVSlice.get / VCFSlice.get
 *                      (formats/generic/csv.py:52-105, formats/genomics/vcf.py:88-149) and the line
 *                      counting gztool does for GZipText/FASTQGZip (formats/compressed/gzipped.py:46-153,
 *                      formats/genomics/fastq.py:19-48), as one sorted offset index (every_k = 4 with
 *                      emit_add = 1 gives FASTQ read end offsets).
 *   dp_find_delim   <- the seek()+readline() that finds the end of a header line cut by a chunk end
 *                      (fasta.py:45-56) — used to resolve ends beyond the bytes a call was given.
 */
#ifndef DPSCAN_H
#define DPSCAN_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DP_OK 0
#define DP_ERR_INVALID 1   /* bad argument */
#define DP_ERR_HIP 2       /* a HIP runtime call failed (message in dp_last_error) */
#define DP_ERR_CAPACITY 3  /* output capacity too small; the required count is still returned */
#define DP_ERR_OVERFLOW 4  /* a uint32 offset would be >= 2^32 (the reference raises OverflowError) */
#define DP_ERR_TIMEOUT 5   /* an inter-workgroup wait hit its bound (kernel terminated, results invalid) */

typedef struct dp_ctx dp_ctx;

/* ABI version history: 1 (rounds 1-4); 2 (round 5): dp_scan_delim_form gained its out_mode argument, dp_scan_forms
   was removed, dp_ctx_set_form / dp_ctx_get_form / dp_last_delim_form were added.  A binding checks
   dp_abi_version() >= DP_ABI_VERSION before it binds anything (dataplug_amd/scan/_lib.py refuses older builds). */
#define DP_ABI_VERSION 2
int dp_abi_version(void);                                  /* returns DP_ABI_VERSION of the build */
const char* dp_last_error(void);                           /* thread-local message of the last failure */
int dp_device_count(int* n);
int dp_ctx_create(int device, dp_ctx** out);               /* binds `device`, creates a non-blocking stream */
int dp_ctx_destroy(dp_ctx* ctx);
int dp_ctx_get_stream(dp_ctx* ctx, void** stream);
int dp_ctx_set_stream(dp_ctx* ctx, void* stream);          /* NULL restores the ctx's own stream */
int dp_ctx_device(dp_ctx* ctx, int* device);
/* Make ctx's stream wait (on the device, no host sync) for everything enqueued so far on other's
 * stream: a device-scope event, so a caller alternating two contexts keeps its scans serialized on
 * the GPU while it collects one result and enqueues the next (bench.py). */
int dp_ctx_wait(dp_ctx* ctx, dp_ctx* other);

int dp_malloc(dp_ctx* ctx, uint64_t bytes, void** dptr);   /* device memory on the ctx's device */
int dp_free(dp_ctx* ctx, void* dptr);
int dp_host_alloc(uint64_t bytes, void** hptr);            /* pinned host memory */
int dp_host_free(void* hptr);
int dp_h2d(dp_ctx* ctx, void* dst, const void* src, uint64_t n);   /* async on the ctx stream */
int dp_d2h(dp_ctx* ctx, void* dst, const void* src, uint64_t n);   /* async on the ctx stream */
int dp_sync(dp_ctx* ctx);                                           /* waits for the ctx stream */

/*
 * FASTA header index (fasta.py:24-74 semantics, bit-exact).
 *   d_buf[0 .. buf_len) holds object bytes [buf_base, buf_base + buf_len); obj_size is the object size.
 *   chunks[2*i], chunks[2*i+1] = [c0, c1) of chunk i in OBJECT offsets (the reference chunk plan, which
 *   may overlap); every chunk must lie inside the buffer.  Per chunk, a '>' at p is a header start iff
 *   p+1 < c1, d[p+1] != '\n' and no earlier '>' lies on the same line inside the chunk; its end is
 *   1 + the first '\n' at or after p in the whole object, or obj_size if there is none.
 *   d_out receives interleaved (start, end) pairs in chunk order, as uint32 (out_u64 = 0, the reference
 *   format) or uint64; at most cap_pairs pairs are written, *n_pairs is the full count.
 *   pending (host array of nchunks, may be NULL): -1, or the pair index whose end lies beyond the
 *   buffer end (buf_base + buf_len < obj_size); resolve those with dp_find_delim on later bytes.
 *   chunk_end (host array of nchunks, may be NULL): pairs emitted up to and including chunk i, so chunk
 *   i owns pairs [chunk_end[i-1], chunk_end[i]) — the per-chunk split merge_fasta_metadata concatenates.
 *   Returns DP_ERR_OVERFLOW when out_u64 = 0 and an offset is >= 2^32.
 */
int dp_fasta_index(dp_ctx* ctx, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base, uint64_t obj_size,
                   const uint64_t* chunks, uint64_t nchunks, void* d_out, int out_u64, uint64_t cap_pairs,
                   uint64_t* n_pairs, int64_t* pending, uint64_t* chunk_end);
/* Same, enqueued without waiting; complete with dp_fasta_result (at most one call in flight per ctx). */
int dp_fasta_index_async(dp_ctx* ctx, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base,
                         uint64_t obj_size, const uint64_t* chunks, uint64_t nchunks, void* d_out, int out_u64,
                         uint64_t cap_pairs);
int dp_fasta_result(dp_ctx* ctx, uint64_t* n_pairs, int64_t* pending, uint64_t* chunk_end);

/*
 * Delimiter offset index over object bytes [begin, end) (object offsets, inside the buffer).
 *   Counting every byte == delim as g = 0, 1, 2, ... in order, the entries with g % every_k == every_k-1
 *   are written as d_out[g / every_k] = offset + emit_add (uint32 if out_u64 = 0 else uint64).
 *   every_k = 1, emit_add = 0: the '\n' offsets of a CSV/VCF body.  every_k = 4, emit_add = 1: FASTQ
 *   read end offsets.  *n_out = entries (full count even beyond cap), *n_delims = delimiters seen.
 */
int dp_delim_index(dp_ctx* ctx, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base, uint64_t begin,
                   uint64_t end, uint32_t delim, uint32_t every_k, uint32_t emit_add, void* d_out, int out_u64,
                   uint64_t cap, uint64_t* n_out, uint64_t* n_delims);
int dp_delim_index_async(dp_ctx* ctx, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base, uint64_t begin,
                         uint64_t end, uint32_t delim, uint32_t every_k, uint32_t emit_add, void* d_out,
                         int out_u64, uint64_t cap);
int dp_delim_result(dp_ctx* ctx, uint64_t* n_out, uint64_t* n_delims);
/*
 * General form: ascending, non-overlapping object ranges ranges[2*i] .. ranges[2*i+1] (inside the buffer)
 * scanned as ONE delimiter stream whose ordinals start at `carry` (the delimiters before the first range,
 * e.g. of the pieces of an inflated stream already indexed), so every_k selection continues across
 * launches: entries are the g with (carry + g) % every_k == every_k - 1, written from d_out[0]; *n_out =
 * (carry + n_delims) / every_k - carry / every_k.
 *   out_mode 0: uint32 (DP_ERR_OVERFLOW at >= 2^32), 1: uint64, 2: uint32 low words (a paged index: split the
 *   ranges at multiples of 2^32 and read each page's first entry from range_end).
 *   out_mode 3: uint16 low words plus a 64 KiB block table -- the stored CSV/VCF index (<key>.lines and
 *   <key>.lines.blocks), a quarter of the uint64 index's bytes:
 *     - every_k must be 1 and emit_add 0 (DP_ERR_INVALID otherwise): every delimiter is an entry, so the
 *       table's delimiter counts are entry indexes, and each low word locates its own byte;
 *     - d_out[0 .. n_out) are uint16: entry i = offset_i & 0xFFFF;
 *     - the block table follows at byte offset (2 * cap + 15) & ~15 of d_out: uint64 tab[j] for
 *       j = 0 .. J-1, J = ((last - 1) >> 16) - j0 + 1 (1 if last == first), j0 = first >> 16, where first =
 *       ranges[0] and last = ranges[2 * nranges - 1]; tab[j] = entries (relative to this launch) before
 *       object offset (j0 + j) << 16, so entry i's full offset is ((j0 + j) << 16) + low word for the j
 *       with tab[j] <= i < tab[j + 1] (tab is non-decreasing).  When `first` is not a multiple of 64 KiB,
 *       tab[0] stands for a boundary below the first byte and is not written: read it as 0.
 *     - d_out must be 16-byte aligned and hold (2 * cap + 15) & ~15 + 8 * J bytes;
 *     - ranges must be contiguous (range i + 1 starts where range i ends), and d_buf and buf_base must be
 *       congruent mod 16 (the kernel's 16-byte lanes then sit on object-aligned 64 KiB boundaries).
 *   out_mode 4: uint8 low bytes, the low 16 bits of the entries before every 256-byte boundary, and the 64 KiB block
 *   table -- an eighth of the uint64 index's bytes plus 2 B per 256 input bytes (round 5's stored CSV/VCF index:
 *   <key>.lines, <key>.lines.sub, <key>.lines.blocks).  Same requirements as out_mode 3, and:
 *     - d_out[0 .. n_out) are uint8: entry i = offset_i & 0xFF;
 *     - the block table (as out_mode 3) at byte offset (cap + 15) & ~15 of d_out;
 *     - then, at byte offset (((cap + 15) & ~15) + 8 * J + 15) & ~15, uint16 sub[s] for s = 0 .. S-1,
 *       S = ((last - 1) >> 8) - s0 + 1 (1 if last == first), s0 = first >> 8: sub[s] = (entries before object offset
 *       (s0 + s) << 8) & 0xFFFF.  Within a 64 KiB block the counts before its 256-byte boundaries exceed the block's
 *       tab entry by less than 2^16, so the full count is tab[j] + ((sub[s] - tab[j]) mod 2^16) for the block j
 *       holding the boundary, and entry i's offset is ((s0 + s) << 8) + low byte for the s with
 *       count(s) <= i < count(s + 1).  When `first` is not a multiple of 256, sub[0] stands for a boundary below the
 *       first byte and is not written: read it as 0;
 *     - d_out must hold that offset + 2 * S bytes.
 *   range_end (host array of nranges, may be NULL): delimiters up to and including range i.
 */
int dp_delim_ranges_async(dp_ctx* ctx, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base,
                          const uint64_t* ranges, uint64_t nranges, uint32_t delim, uint32_t every_k,
                          uint32_t emit_add, uint64_t carry, void* d_out, int out_mode, uint64_t cap);
int dp_delim_ranges_result(dp_ctx* ctx, uint64_t* n_out, uint64_t* n_delims, uint64_t* range_end);

/* First object offset >= from holding `delim` in the buffer, or -1 (seek+readline of fasta.py:45-56). */
int dp_find_delim(dp_ctx* ctx, const uint8_t* d_buf, uint64_t buf_len, uint64_t buf_base, uint64_t from,
                  uint32_t delim, int64_t* pos);

/* Calibration (async, timed like the scans): read `bytes` (16-byte multiple) once with the best plain
 * streaming kernel measured (the read-only ceiling next to the roofline fraction); dp_stream_rw also writes
 * write_q16 / 65536 output bytes per input byte (contiguous non-temporal runs, one per workgroup step of 16
 * ranges of 16 KiB; whole 16 KiB ranges only), the newline index's traffic mix: a same-run reference for it,
 * not a bound.  blocks_per_cu <= 0: one 1024-thread workgroup per CU.  Like the scans, they run on the
 * device's scan stream, so within a process they never overlap a scan (another process's grids still may). */
int dp_stream_read(dp_ctx* ctx, const void* d_buf, uint64_t bytes, int blocks_per_cu);
int dp_stream_rw(dp_ctx* ctx, const void* d_in, uint64_t bytes, void* d_out, uint32_t write_q16, int blocks_per_cu);

/* Kernel timing (off by default): HIP events around every scan launch -- on the device's scan stream,
 * around the scan's kernels alone (FASTA: the map and placement kernels as one span) -- and around the
 * calibration kernels on the ctx stream. */
int dp_timing_enable(dp_ctx* ctx, int enable);
int dp_timing_read(dp_ctx* ctx, double* total_ms, uint64_t* launches);   /* syncs; then resets */

/* Diagnostics: the realtime stamps of the last scan launch (map_kernel per wave, fasta_place_kernel per block,
 * line_kernel per step; `slots` words per wave, `waves` waves per workgroup).  Only the diagnostics build
 * (-DDP_DIAG, lib/libdpscan_diag.so) records them; the shipped library returns DP_ERR_INVALID. */
int dp_debug_profile(dp_ctx* ctx, uint64_t* host_words, uint64_t n_words, int* slots, int* waves);

/* Device (hipMalloc) and pinned host (hipHostMalloc) allocations the library has made in this process so
 * far: dp_malloc / dp_host_alloc and every context's own workspace (chunk table, look-back descriptors,
 * FASTA range summaries and spill).  Steady-state calls on warm contexts allocate nothing. */
int dp_alloc_counts(uint64_t* device_allocs, uint64_t* host_allocs);

/* The kernels a ctx's scans take.  The defaults are the shipped choices; a library reads no environment
 * variable, so only these calls change them (tests and same-box A/B runs):
 *   DP_FORM_FASTA           0 = map + placement kernels (default), 1 = the one-pass look-back kernel;
 *   DP_FORM_DELIM           0 = auto (default), 1 = line_kernel (lockstep one pass), 3 = the one-pass look-back
 *                           kernel, at every launch size (2, round 3's map + placement form, was removed in round 5);
 *   DP_FORM_DELIM_LINE_MAX  auto: launches of up to this many bytes (the sum of the ranges) run line_kernel
 *                           (default 4 GiB);
 *   DP_FORM_DELIM_DENSE     auto, above that size (out_mode 0-3): a density probe kernel counts the delimiters of
 *                           256 KiB sampled evenly from the launch's own bytes and picks line_kernel at this many
 *                           or more delimiters per KiB x 1000 (default 20000: CSV-like), the one-pass kernel below.
 * Every form writes the same output.  Not while a scan is in flight on the ctx. */
#define DP_FORM_FASTA 0
#define DP_FORM_DELIM 1
#define DP_FORM_DELIM_LINE_MAX 2
#define DP_FORM_DELIM_DENSE 3
int dp_ctx_set_form(dp_ctx* ctx, int what, uint64_t value);
int dp_ctx_get_form(dp_ctx* ctx, int what, uint64_t* value);
/* The kernels the ctx's next newline launch scanning `span` bytes into `out_mode` takes: 1 = line_kernel, 3 = the
 * one-pass look-back kernel, 0 = decided on the device from the launch's bytes (auto above DP_FORM_DELIM_LINE_MAX;
 * out_mode 4, the uint8 index, runs line_kernel at every size under auto). */
int dp_scan_delim_form(dp_ctx* ctx, uint64_t span, int out_mode, int* form);
/* The kernels the ctx's last collected newline launch ran (1 or 3; 0 before any): the probe's pick read back
 * with the launch's results. */
int dp_last_delim_form(dp_ctx* ctx, int* form);

/* Launch geometry (for tests/tuning): workgroups of the persistent scan grid, and unit size in bytes. */
int dp_scan_geometry(dp_ctx* ctx, int* grid, int* unit_bytes);

#ifdef __cplusplus
}
#endif
#endif /* DPSCAN_H */
