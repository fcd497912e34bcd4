"""Object-level index builds: storage → pinned host → HBM → HIP scan → host index.

These are what the format plugins call.  Everything computational runs in libdpscan (HIP); the host side
only moves bytes and stitches per-GPU results in chunk order.  Multi-GPU: an object's map chunks are
independent (preprocess.py:39-51 of the reference), so the chunk list is cut into contiguous groups, one
per GPU, each scanned by one launch on its own device; no collective.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import threading
from dataclasses import dataclass
from functools import partial
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ._lib import DPCapacityError, DPScanUnavailable
from ..dist import split_groups
from ..storage.ranges import GET_PART as _GET_PART, GET_THREADS as _GET_THREADS, read_range_into
from .device import close_context, ScanContext, device_count, get_context

_HALO0 = 64 << 10             # first look-ahead window when a header line crosses the fetched bytes
# HBM one FASTA launch may hold: a GPU's chunk group whose bytes plus scan workspace exceed this (an object far
# beyond 288 GB x GPUs, or a small budget set for tests) is scanned in several passes of whole chunks
MAX_LAUNCH_BYTES = 64 << 30
# the FASTA scan's workspace per input byte (libdpscan ensure_ranges): a 16-byte range record and a 1 KiB spill
# slot per 16 KiB range, grown with 1/8 headroom -- 7.1 % on top of the input bytes
WORKSPACE_PER_BYTE = (16 + 512 * 2) / 16384 * 1.125


def max_launch_bytes() -> int:
    """Input bytes one launch may span: the HBM budget (``DATAPLUG_AMD_MAX_LAUNCH_BYTES``) less the workspace
    the scan allocates for them."""
    budget = int(os.environ.get("DATAPLUG_AMD_MAX_LAUNCH_BYTES", MAX_LAUNCH_BYTES))
    return max(1, int(budget / (1.0 + WORKSPACE_PER_BYTE)))


DEVICES_ATTR = "_dataplug_devices"


def parse_devices(spec) -> Optional[List[int]]:
    """A device list from ``parallel_config["dataplug_devices"]`` / ``extra_args["dataplug_devices"]``
    (an int count, a list of ordinals, or a "0,1,..." string); None if unset.  Repeating an ordinal runs
    several groups on one GPU (how the multi-GPU split is rehearsed on a 1-GPU box)."""
    if spec is None:
        return None
    if isinstance(spec, str):
        devs = [int(x) for x in spec.split(",") if x.strip()]
    elif isinstance(spec, int) and not isinstance(spec, bool):
        if spec <= 0:
            raise ValueError(f"dataplug_devices={spec}: need at least one GPU")
        devs = list(range(spec))
    else:
        devs = [int(x) for x in spec]
    if not devs or any(d < 0 for d in devs):
        raise ValueError(f"dataplug_devices={spec!r}: expected a non-empty list of GPU ordinals")
    return devs


def devices(max_devices: Optional[int] = None, co=None) -> List[int]:
    """GPUs an index build runs on: the object's ``dataplug_devices`` (set by ``co.preprocess`` from its
    ``parallel_config`` / ``extra_args``), else ``DATAPLUG_AMD_DEVICES``, else every visible GPU."""
    env = os.environ.get("DATAPLUG_AMD_DEVICES")
    own = getattr(co, DEVICES_ATTR, None) if co is not None else None
    if own:
        devs = list(own)
    elif env:
        devs = [int(x) for x in env.split(",") if x.strip()]
    else:
        n = device_count()
        if n <= 0:
            raise DPScanUnavailable("no HIP device visible: the index build runs on MI355X GPUs only")
        devs = list(range(n))
    return devs[:max_devices] if max_devices else devs


# ------------------------------------------------------------------------------------------ storage → host
def fetch_to_device(ctx: ScanContext, storage, bucket: str, key: str, lo: int, hi: int, d_ptr: int,
                    part: Optional[int] = None, threads: int = _GET_THREADS, staging: str = "object"):
    """Object bytes [lo, hi) into device memory at ``d_ptr``: parallel ranged GETs into the context's pinned
    staging buffer, each part's H2D copy issued on the context stream as soon as that part has landed, so
    the PCIe copy overlaps the remaining GETs (storage -> pinned -> HBM pipeline).
    Returns the pinned buffer (valid until the context's next fetch).  The copies are asynchronous: work
    enqueued afterwards on the same stream (the scan) sees the bytes."""
    n = hi - lo
    part = part or _GET_PART
    host = ctx.pinned(staging, max(n, 1))
    if n <= 0:
        return host
    if n <= part:
        read_range_into(storage, bucket, key, lo, hi, host.view(n), part=part, threads=threads)
        ctx.h2d_async(d_ptr, host.ptr, n)
        return host
    land_gets(ctx, submit_gets(ctx.get_pool(threads), storage, bucket, key, lo, hi, host, part), d_ptr)
    return host


def submit_gets(pool, storage, bucket: str, key: str, lo: int, hi: int, host, part: int = _GET_PART):
    """Queue the ranged GETs of object bytes [lo, hi) into pinned ``host`` on ``pool`` (parts of ``part`` bytes, in
    order); ``land_gets`` copies them to the device as they land.  Queued behind another fetch's GETs on the same
    pool, they start as its last ones finish (a continuous GET stream across pieces)."""
    n = hi - lo
    view = host.view(n)

    def one(a: int) -> int:
        read_range_into(storage, bucket, key, lo + a, lo + min(n, a + part), view[a:], part=part, threads=1)
        return a
    return host, n, part, [pool.submit(one, a) for a in range(0, n, part)]


def land_gets(ctx: ScanContext, gets, d_ptr: int) -> None:
    """Each part of ``submit_gets`` copied to ``d_ptr`` on the context stream as soon as it lands (H2D issued from
    the calling thread only); a failed GET cancels the rest, and none may still land in the staging buffer."""
    host, n, part, futs = gets
    try:
        for f in cf.as_completed(futs):
            a = f.result()
            ctx.h2d_async(d_ptr + a, host.ptr + a, min(n, a + part) - a)
    except BaseException:
        cancel_gets(gets)
        raise


def cancel_gets(gets) -> None:
    for f in gets[3]:
        f.cancel()
    cf.wait(gets[3])


def resolve_line_end(ctx: ScanContext, storage, bucket: str, key: str, size: int, pos: int) -> int:
    """1 + the first '\\n' at or after object offset ``pos``, or ``size`` (what the reference's
    seek(start) + readline() + tell() gives for a header cut by its chunk end, fasta.py:45-56).
    The search itself runs on the GPU (dp_find_delim) over growing look-ahead windows."""
    win = _HALO0
    while pos < size:
        hi = min(size, pos + win)
        buf = ctx.pinned("halo", hi - pos)
        read_range_into(storage, bucket, key, pos, hi, buf.view(hi - pos))
        d = ctx.workspace("halo", hi - pos + 64)
        ctx.h2d_async(d.ptr, buf.ptr, hi - pos)
        p = ctx.find_delim(d.ptr, hi - pos, pos, pos, 10)
        if p >= 0:
            return p + 1
        pos = hi
        win *= 4
    return size


# ------------------------------------------------------------------------------------------ per-GPU workers
_workers_lock = threading.Lock()
_workers = {}


def group_worker(device: int, slot: int = 0) -> cf.ThreadPoolExecutor:
    """The long-lived worker thread of (device, slot): a one-thread executor whose thread keeps its
    ``ScanContext`` — stream, pinned staging and HBM workspace — across calls, so a multi-GPU
    ``co.preprocess`` allocates nothing once its buffers have grown to the object size.  ``slot`` tells
    apart several groups on one device (``dataplug_devices=[0, 0]``, the one-GPU rehearsal of the split)."""
    key = (int(device), int(slot))
    with _workers_lock:
        ex = _workers.get(key)
        if ex is None:
            ex = _workers[key] = cf.ThreadPoolExecutor(1, thread_name_prefix=f"dpscan-gpu{device}.{slot}")
        return ex


def release_workers() -> None:
    """Free what every persistent worker holds: each closes its thread's contexts (pinned staging, HBM
    workspace, stream), which its next job recreates.  For a process that indexed one very large object and goes
    on with other work."""
    with _workers_lock:
        items = list(_workers.items())
    for (dev, _), ex in items:
        ex.submit(close_context, dev).result()


def run_on_devices(devs: Sequence[int], jobs: Sequence) -> list:
    """Run job k (a callable taking no argument) on device devs[k]'s persistent worker; one job alone runs
    on the calling thread (its own thread-local context).  Returns the results in job order."""
    if len(jobs) == 1:
        return [jobs[0]()]
    seen = {}
    futs = []
    for k, job in enumerate(jobs):
        d = devs[k]
        slot = seen.get(d, 0)
        seen[d] = slot + 1
        futs.append(group_worker(d, slot).submit(job))
    return [f.result() for f in futs]


# ------------------------------------------------------------------------------------------ FASTA
@dataclass(frozen=True)
class FastaGroup:
    """One GPU's share of a FASTA scan plan: entries [i0, i1) of the plan (contiguous, so the outputs
    concatenate in chunk order like merge_fasta_metadata, fasta.py:66-74), the bytes they scan [lo, hi),
    and the bytes fetched into HBM [lo, buf_hi): ``hi`` plus a look-ahead halo, so a header line cut by the
    group's last chunk usually ends inside the same launch (resolve kernel) instead of a later GET."""
    i0: int
    i1: int
    lo: int
    hi: int
    buf_hi: int

    def chunks(self, plan: Sequence[Tuple[int, int]]) -> List[Tuple[int, int]]:
        return list(plan[self.i0:self.i1])


@dataclass(frozen=True)
class FastaPiece:
    """Bytes [a, b) of chunk ``chunk`` of the reference's plan, scanned as one launch chunk [a, end).  A
    piece cut inside its chunk scans one byte past its end (end = b + 1): a '>' at b - 1 is then judged with
    its next byte, as in the whole chunk (fasta.py:36 needs p + 1 < chunk end), while a '>' at b itself is
    left to the next piece.  ``first``: a is the chunk's own start (the line state starts empty there)."""
    chunk: int
    a: int
    b: int
    end: int
    first: bool


def fasta_pieces(plan: Sequence[Tuple[int, int]], n_groups: int) -> List[List[FastaPiece]]:
    """The reference's chunk plan cut into ``n_groups`` byte-balanced, contiguous runs of pieces (SURVEY.md
    §8(e)).  Group boundaries fall at every total/n bytes of chunk data, so a plan with fewer chunks than
    GPUs (the reference's canonical ``chunk_size = ceil(size / 4)`` on 8 GPUs) still fills every GPU; a
    boundary within ``snap`` bytes of a chunk boundary moves there (no sliver pieces), so an equal-chunk plan
    whose chunk count the group count divides is not cut at all."""
    n_groups = max(1, int(n_groups))
    lens = [max(0, c1 - c0) for c0, c1 in plan]
    total = sum(lens)
    starts = np.concatenate(([0], np.cumsum(lens, dtype=np.int64))) if plan else np.zeros(1, np.int64)
    targets = sorted({(k * total) // n_groups for k in range(1, n_groups)} - {0, total}) if total else []
    snap = min(1 << 20, total // (8 * n_groups)) if total else 0
    bounds = []                                          # cumulative byte positions of the group boundaries
    for t in targets:
        i = int(np.searchsorted(starts, t, side="right")) - 1        # chunk holding byte t
        near = min((int(starts[i]), int(starts[i + 1])), key=lambda x: abs(x - t)) if i + 1 < len(starts) else t
        bounds.append(near if abs(near - t) <= snap else t)
    bounds = sorted(set(b for b in bounds if 0 < b < total))
    groups: List[List[FastaPiece]] = [[] for _ in range(len(bounds) + 1)]
    for i, (c0, c1) in enumerate(plan):
        s0, s1 = int(starts[i]), int(starts[i] + lens[i])
        cuts = [b for b in bounds if s0 < b < s1]
        edges = [s0] + cuts + [s1]
        for j in range(len(edges) - 1):
            a = c0 + (edges[j] - s0)
            b = c0 + (edges[j + 1] - s0)
            last = j == len(edges) - 2
            g = int(np.searchsorted(np.asarray(bounds, np.int64), edges[j], side="right"))
            groups[g].append(FastaPiece(i, a, b, b if last else b + 1, j == 0))
    return [g for g in groups if g]


def fasta_split(plan: Sequence[Tuple[int, int]], n_groups: int, size: int, halo: int = _HALO0):
    """(pieces, scan plan, groups): ``fasta_pieces`` flattened in order, the launch chunks ``[(a, end)]`` of
    those pieces, and one ``FastaGroup`` per GPU over that scan plan.  Used by ``fasta_index_object`` and by
    bench.py's multi-GPU line (one thread or rank per group)."""
    runs = fasta_pieces(plan, n_groups)
    pieces = [p for r in runs for p in r]
    scan_plan = [(p.a, p.end) for p in pieces]
    groups, i = [], 0
    for r in runs:
        j = i + len(r)
        lo = min(p.a for p in r)
        hi = max(p.end for p in r)
        groups.append(FastaGroup(i, j, lo, hi, min(size, hi + halo)))
        i = j
    return pieces, scan_plan, groups


def fasta_groups(plan: Sequence[Tuple[int, int]], n_groups: int, size: int, halo: int = _HALO0) -> List[FastaGroup]:
    """The multi-GPU split of one object's chunk plan when its chunks are kept whole: ``split_groups`` of the
    chunk list over ``n_groups`` GPUs (tests/test_dist_gloo.py's reference split)."""
    out = []
    for i0, i1 in split_groups(len(plan), n_groups):
        if i1 <= i0:
            continue
        lo = min(c0 for c0, _ in plan[i0:i1])
        hi = max(c1 for _, c1 in plan[i0:i1])
        out.append(FastaGroup(i0, i1, lo, hi, min(size, hi + halo)))
    return out


def fasta_passes(plan: Sequence[Tuple[int, int]], g: FastaGroup, size: int, budget: int,
                 halo: int = _HALO0) -> List[FastaGroup]:
    """``g`` cut into consecutive runs of whole chunks whose bytes span at most ``budget`` (a chunk larger
    than the budget is a pass of its own).  Chunks are independent (preprocess.py:39-51), so the passes'
    pairs concatenate in chunk order like the groups' do."""
    if g.buf_hi - g.lo <= budget:
        return [g]
    out = []
    i = g.i0
    while i < g.i1:
        lo, hi = plan[i]
        j = i + 1
        while j < g.i1:
            nlo, nhi = min(lo, plan[j][0]), max(hi, plan[j][1])
            if min(size, nhi + halo) - nlo > budget:
                break
            lo, hi = nlo, nhi
            j += 1
        out.append(FastaGroup(i, j, lo, hi, min(size, hi + halo)))
        i = j
    return out


def _fasta_group(dev: int, co, scan_plan: Sequence[Tuple[int, int]], pieces: Sequence[FastaPiece], g: FastaGroup,
                 u64: bool):
    """One GPU's group on the calling thread's context for ``dev``: (pairs of each piece, first '\\n' of each
    piece cut inside its chunk, or None when it has none)."""
    ctx = get_context(dev)
    size = co.size
    per_piece, first_nl = [], {}
    for p_ in fasta_passes(scan_plan, g, size, max_launch_bytes()):
        n = p_.buf_hi - p_.lo
        d = ctx.workspace("input", n + 64, placed=True)
        fetch_to_device(ctx, co.storage, co.path.bucket, co.path.key, p_.lo, p_.buf_hi, d.ptr)
        pairs, pending, cend = ctx.fasta_index(d.ptr, n, p_.lo, size, p_.chunks(scan_plan), u64=u64)
        for p in pending[pending >= 0]:
            start = int(pairs[p, 0])
            end = resolve_line_end(ctx, co.storage, co.path.bucket, co.path.key, size, p_.buf_hi)
            if not u64 and end > 0xFFFFFFFF:
                raise OverflowError(f"FASTA offset {end} does not fit the uint32 index (header at {start})")
            pairs[p, 1] = end
        prev = 0
        for k in range(p_.i0, p_.i1):
            e = int(cend[k - p_.i0])
            per_piece.append(pairs[prev:e])
            prev = e
            pc = pieces[k]
            if not pc.first:                              # the first line segment of a cut piece
                nl = ctx.find_delim(d.ptr, n, p_.lo, pc.a, 10)
                first_nl[k] = nl if 0 <= nl < pc.end else None
    return per_piece, first_nl


def stitch_pieces(pieces: Sequence[FastaPiece], per_piece: Sequence[np.ndarray], first_nl: dict) -> np.ndarray:
    """Pairs of cut chunks as the whole chunks give them (fasta.py:24-56).  Each piece was scanned with an
    empty line state at its start; where the chunk's true state there says a header is open on the current
    line (the previous piece ended inside a header line), the piece's headers in its first line segment —
    before its first '\\n' — are not headers of the chunk: they are dropped.  The open header's end needs no
    fix: ends are always the object's next '\\n' (resolved on the device or from later bytes).  The state
    carried on is the piece's own at its end (a header pending there) once the piece holds a '\\n', or stays
    open through a piece without one."""
    out = []
    S = False
    for k, (pc, pairs) in enumerate(zip(pieces, per_piece)):
        if pc.first:
            S = False
        pend = len(pairs) > 0 and int(pairs[-1, 1]) > pc.end
        if pc.first:
            keep = pairs
        else:
            nl = first_nl.get(k)
            if S:
                keep = pairs[:0] if nl is None else pairs[pairs[:, 0] > nl]
            else:
                keep = pairs
            if nl is None:
                pend = S or pend
        S = pend
        out.append(keep)
    return np.concatenate(out) if out else np.zeros((0, 2), np.uint32)


def fasta_index_object(co, plan: Sequence[Tuple[int, int]], u64: bool = False,
                       max_devices: Optional[int] = None) -> np.ndarray:
    """(n, 2) (start, end) pairs of every chunk of ``plan`` concatenated in chunk order — the index
    ``merge_fasta_metadata`` (fasta.py:66-74) assembles from the per-chunk map outputs.  The plan's bytes are
    cut into one byte-balanced group per GPU (``fasta_split``), each scanned by its device's persistent
    worker, and the cut chunks are stitched (``stitch_pieces``)."""
    dt = np.uint64 if u64 else np.uint32
    if not plan:
        return np.zeros((0, 2), dt)
    devs = devices(max_devices, co)
    pieces, scan_plan, groups = fasta_split(plan, len(devs), co.size)
    jobs = [partial(_fasta_group, devs[k], co, scan_plan, pieces, g, u64) for k, g in enumerate(groups)]
    per_piece, first_nl = [], {}
    for pp, fn in run_on_devices(devs, jobs):
        first_nl.update(fn)
        per_piece.extend(pp)
    return stitch_pieces(pieces, per_piece, first_nl).astype(dt, copy=False)


def fasta_index_chunk(co, data, chunk_offset: int, job: int = 0, u64: bool = False) -> np.ndarray:
    """Pairs of one map chunk whose bytes ``data`` the caller already holds (the per-chunk plugin call),
    scanned on GPU ``job % n_gpus``."""
    devs = devices(co=co)
    ctx = get_context(devs[job % len(devs)])
    n = len(data)
    pairs, pending, _ = ctx.fasta_index_host(data, chunk_offset, co.size, [(chunk_offset, chunk_offset + n)], u64=u64)
    for p in pending[pending >= 0]:
        end = resolve_line_end(ctx, co.storage, co.path.bucket, co.path.key, co.size, chunk_offset + n)
        if not u64 and end > 0xFFFFFFFF:
            raise OverflowError(f"FASTA offset {end} does not fit the uint32 index")
        pairs[p, 1] = end
    return pairs


# ------------------------------------------------------------------------------------------ newline / record index
PAGE = 1 << 32


def page_ranges(lo: int, hi: int) -> List[Tuple[int, int]]:
    """[lo, hi) split at multiples of 2^32: the ranges of a paged (uint32 low word) newline index."""
    out, p = [], lo
    while p < hi:
        q = min(hi, (p // PAGE + 1) * PAGE)
        out.append((p, q))
        p = q
    return out


@dataclass
class PagedOffsets:
    """Sorted object offsets as uint32 low words plus, for every 4 GiB page boundary p * 2^32 (p >= 1) below
    the end of the scanned bytes, the number of offsets before it: offset i = (page(i) << 32) | low[i] with
    page(i) = bisect_right(pages, i).  Half the bytes of a uint64 index, written by the GPU directly
    (dp_delim_ranges out_mode 2), at the same information."""
    low: np.ndarray
    pages: List[int]

    def __len__(self) -> int:
        return len(self.low)

    def to_u64(self, i0: int = 0, i1: Optional[int] = None) -> np.ndarray:
        i1 = len(self.low) if i1 is None else i1
        idx = np.arange(i0, i1, dtype=np.int64)
        page = np.searchsorted(np.asarray(self.pages, np.int64), idx, side="right").astype(np.uint64)
        return (page << np.uint64(32)) | self.low[i0:i1].astype(np.uint64)


@dataclass
class BlockedOffsets:
    """Sorted object offsets as uint16 low words plus a table of the entries before every 64 KiB boundary:
    offset i = ((j0 + j) << 16) | low[i] with j = bisect_right(table, i) - 1, table[0] = 0 (the boundary at
    or below the first byte).  A quarter of the bytes of a uint64 index (for a 64 GiB object the table is
    8 MiB), written by the GPU directly (dp_delim_ranges out_mode 3)."""
    low: np.ndarray
    table: np.ndarray
    j0: int

    def __len__(self) -> int:
        return len(self.low)

    def to_u64(self, i0: int = 0, i1: Optional[int] = None) -> np.ndarray:
        i1 = len(self.low) if i1 is None else i1
        idx = np.arange(i0, i1, dtype=np.int64)
        blk = np.searchsorted(self.table.astype(np.int64), idx, side="right").astype(np.uint64) - np.uint64(1)
        return ((blk + np.uint64(self.j0)) << np.uint64(16)) | self.low[i0:i1].astype(np.uint64)


def sub_counts(sub: np.ndarray, table: np.ndarray, s0: int, j0: int, sa: int = 0) -> np.ndarray:
    """Entries before each 256-byte boundary (s0 + sa + i) << 8 of a uint8 index, as uint64: the block table's count
    at the boundary's 64 KiB block plus the 16-bit difference the sub-block table holds (a 64 KiB block's 256
    boundaries differ from its first by less than 2^16 entries)."""
    s = np.arange(sa, sa + len(sub), dtype=np.int64)
    base = table[((s0 + s) >> 8) - j0].astype(np.uint64)
    return base + ((sub.astype(np.uint64) - base) & np.uint64(0xFFFF))


@dataclass
class ByteOffsets:
    """Sorted object offsets as uint8 low bytes, a table of the entries before every 256-byte boundary (their low
    16 bits) and the 64 KiB block table: offset i = ((s0 + s) << 8) | low[i] with s = bisect_right(C, i) - 1, C the
    counts before the 256-byte boundaries (``sub_counts``), table[0] / sub[0] = 0 for the boundaries at or below the
    first byte.  An eighth of the bytes of a uint64 index plus 2 B per 256 input bytes, written by the GPU directly
    (dp_delim_ranges out_mode 4)."""
    low: np.ndarray
    sub: np.ndarray
    table: np.ndarray
    s0: int
    j0: int

    def __len__(self) -> int:
        return len(self.low)

    def to_u64(self, i0: int = 0, i1: Optional[int] = None) -> np.ndarray:
        i1 = len(self.low) if i1 is None else i1
        c = sub_counts(self.sub, self.table, self.s0, self.j0)
        idx = np.arange(i0, i1, dtype=np.uint64)
        s = np.searchsorted(c, idx, side="right").astype(np.uint64) - np.uint64(1)
        return ((s + np.uint64(self.s0)) << np.uint64(8)) | self.low[i0:i1].astype(np.uint64)


INDEX_FORMATS = ("u8s", "u16b", "u32p", "u64")
# "auto" (the CSV / VCF plugins' default): u8s costs 1 B per entry + 2 B per 256 object bytes, u16b 2 B per entry
# (both + 8 B per 64 KiB), so u8s is the smaller index and the cheaper read while there is a delimiter at least
# every 128 bytes; sparser objects (multi-sample VCF rows of 100 KB) store u16b.
AUTO_BYTES_PER_ENTRY = 128
_AUTO_SAMPLES, _AUTO_SAMPLE_BYTES = 8, 64 << 10


def line_index_form(co, begin: int, end: int, delim: int = 10) -> str:
    """The stored form "auto" picks for object bytes [begin, end): u8s unless a sample of the object (8 ranged GETs
    of 64 KiB spread evenly; the whole range when it is smaller) holds fewer than one delimiter per
    ``AUTO_BYTES_PER_ENTRY`` bytes.  Either form stores the same offsets; this only sizes the index."""
    n = end - begin
    if n <= 0:
        return "u8s"
    if n <= _AUTO_SAMPLES * _AUTO_SAMPLE_BYTES:
        spans = [(begin, end)]
    else:
        step = (n - _AUTO_SAMPLE_BYTES) // (_AUTO_SAMPLES - 1)
        spans = [(begin + k * step, begin + k * step + _AUTO_SAMPLE_BYTES) for k in range(_AUTO_SAMPLES)]
    def sample(span):
        a, b = span
        raw = co.storage.get_object(Bucket=co.path.bucket, Key=co.path.key, Range=f"bytes={a}-{b - 1}")["Body"].read()
        return len(raw), raw.count(bytes([delim]))
    if len(spans) == 1:
        got = [sample(spans[0])]
    else:
        with cf.ThreadPoolExecutor(len(spans)) as ex:      # one round trip, not eight
            got = list(ex.map(sample, spans))
    seen, hits = sum(g[0] for g in got), sum(g[1] for g in got)
    return "u8s" if hits * AUTO_BYTES_PER_ENTRY >= seen else "u16b"


def line_parts(begin: int, end: int, n_devices: int, part_bytes: int = 16 << 30) -> List[Tuple[int, int]]:
    """Raw byte parts of [begin, end) for a newline index (at most ``part_bytes`` each, at least one per
    GPU); part k runs on GPU k mod n_devices and the parts' offsets concatenate to the whole index."""
    if end <= begin:
        return []
    nparts = max(n_devices, -(-(end - begin) // part_bytes))
    step = -(-(end - begin) // nparts)
    bounds = [(begin + i * step, min(end, begin + (i + 1) * step)) for i in range(nparts)]
    return [b for b in bounds if b[1] > b[0]]


def _delim_group(dev: int, co, lo: int, hi: int, delim: int, every_k: int, emit_add: int, fmt: str = "u64"):
    ctx = get_context(dev)
    n = hi - lo
    d = ctx.workspace("input", n + 64, placed=True)
    dp = d.ptr + (lo & 15)                # object offset and device address congruent mod 16 (out_mode 3 grid)
    fetch_to_device(ctx, co.storage, co.path.bucket, co.path.key, lo, hi, dp)
    if fmt == "u64":
        return ctx.delim_index(dp, n, lo, lo, hi, delim=delim, every_k=every_k, emit_add=emit_add, u64=True)
    if fmt == "u32p":
        rg = page_ranges(lo, hi)
        low, nd, ends = ctx.delim_ranges(dp, n, lo, rg, delim=delim, out_mode=2)
        return low, [(r, int(e)) for r, e in zip(rg, ends)]
    if fmt == "u8s":
        low, nd, ends, tab, sub = ctx.delim_ranges(dp, n, lo, [(lo, hi)], delim=delim, out_mode=4)
        return low, tab, sub
    low, nd, ends, tab = ctx.delim_ranges(dp, n, lo, [(lo, hi)], delim=delim, out_mode=3)
    return low, tab


def line_index_object(co, begin: int = 0, end: Optional[int] = None, delim: int = 10,
                      max_devices: Optional[int] = None, part_bytes: int = 8 << 30, fmt: str = "u64"):
    """Sorted offsets of every ``delim`` byte of object bytes [begin, end) in one of ``INDEX_FORMATS``:
    ``u64`` a uint64 array; ``u32p`` a ``PagedOffsets`` (uint32 low words + 4 GiB page counts); ``u16b`` a
    ``BlockedOffsets`` (uint16 low words + a 64 KiB block table); ``u8s`` a ``ByteOffsets`` (uint8 low bytes + the
    256-byte counts + the 64 KiB block table) — the GPU writes 8, 4, 2 or 1 bytes per offset; ``auto`` u8s or
    u16b by the object's delimiter density (``line_index_form``).

    The range is cut into independent parts (at most ``part_bytes`` each, at least one per GPU) scanned
    round-robin on the GPUs and concatenated in order.  The default 8 GiB parts fit an input buffer the context
    allocates placement-aware (``device.PLACEMENT_MAX``: larger buffers are not probed)."""
    if fmt != "auto" and fmt not in INDEX_FORMATS:
        raise ValueError(f"index format must be 'auto' or one of {INDEX_FORMATS}, not {fmt!r}")
    end = co.size if end is None else end
    if fmt == "auto":
        fmt = line_index_form(co, begin, end, delim)
    if end <= begin:
        return {"u64": np.zeros(0, np.uint64), "u32p": PagedOffsets(np.zeros(0, np.uint32), []),
                "u16b": BlockedOffsets(np.zeros(0, np.uint16), np.zeros(1, np.uint64), begin >> 16),
                "u8s": ByteOffsets(np.zeros(0, np.uint8), np.zeros(1, np.uint16), np.zeros(1, np.uint64), begin >> 8,
                                   begin >> 16)}[fmt]
    devs = devices(max_devices, co)
    bounds = line_parts(begin, end, len(devs), part_bytes)

    def run(k: int):
        lo, hi = bounds[k]
        r = _delim_group(devs[k % len(devs)], co, lo, hi, delim, 1, 0, fmt=fmt)
        return r[0] if fmt == "u64" else r

    # parts of one device entry run in order on that entry's persistent worker (run_on_devices)
    by_dev = {}
    for k in range(len(bounds)):
        by_dev.setdefault(k % len(devs), []).append(k)
    out = [None] * len(bounds)

    def worker(ks):
        for k in ks:
            out[k] = run(k)

    entries = sorted(by_dev)
    run_on_devices([devs[e] for e in entries], [partial(worker, by_dev[e]) for e in entries])
    if fmt == "u64":
        return out[0] if len(out) == 1 else np.concatenate(out)
    low = out[0][0] if len(out) == 1 else np.concatenate([o[0] for o in out])
    if fmt == "u32p":
        # pages[p - 1] = offsets before p * 2^32: 0 for the boundaries at or below begin, then the running
        # count at every boundary inside (begin, end) — each starts one of the parts' page ranges
        pages, before = [0] * (begin // PAGE), 0
        for _, ranges in out:
            prev = 0
            for (lo, hi), cum in ranges:
                if lo % PAGE == 0 and lo > begin:
                    pages.append(before)
                before += cum - prev
                prev = cum
        return PagedOffsets(low, pages)
    if len(out) == 1:                                    # one part: [begin, end) itself, its tables as they are
        o = out[0]
        return ByteOffsets(low, o[2], o[1], begin >> 8, begin >> 16) if fmt == "u8s" else \
            BlockedOffsets(low, o[1], begin >> 16)
    merge = PieceMerge(begin, end, fmt)
    pieces = [merge.piece(lo, hi, o) for (lo, hi), o in zip(bounds, out)]
    table = np.concatenate([merge.head_table()] + [p[1] for p in pieces])
    if fmt == "u8s":
        subs = np.concatenate([merge.head_sub()] + [p[2] for p in pieces])
        return ByteOffsets(low, subs, table, merge.S0, merge.J0)
    return BlockedOffsets(low, table, merge.J0)


class PieceMerge:
    """Per-part outputs of a u16b / u8s newline index, in object order, as slices of the whole range's tables.

    table[j - J0] = entries before j * 64 KiB; a boundary inside part k comes from part k's own table (its count
    within the part) plus every earlier part's count; so do u8s's 256-byte counts (low 16 bits, wrapping).  A part's
    boundaries at or after its first byte are all of its table but the first entry when the part starts off a
    boundary, and the whole range's first entry is 0 when ``begin`` is off a boundary (``head_table`` /
    ``head_sub``): slices, no per-entry index arrays (a 16 GiB part has 64 Mi 256-byte counts)."""

    def __init__(self, begin: int, end: int, fmt: str):
        self.begin, self.end, self.fmt = begin, end, fmt
        self.J0, self.S0 = begin >> 16, begin >> 8
        self.before = 0
        self.next_lo = begin

    def head_table(self) -> np.ndarray:
        return np.zeros(1 if self.begin & 0xFFFF else 0, np.uint64)

    def head_sub(self) -> np.ndarray:
        return np.zeros(1 if self.begin & 0xFF else 0, np.uint16)

    def piece(self, lo: int, hi: int, out):
        """(low, table slice, sub slice or None) of part [lo, hi) -- the parts in order, without gaps."""
        if lo != self.next_lo or hi <= lo:
            raise ValueError(f"part [{lo}, {hi}) does not follow [.., {self.next_lo})")
        self.next_lo = hi
        low, tab = out[0], out[1]
        a, b = (lo >> 16) + (1 if lo & 0xFFFF else 0), (hi - 1) >> 16
        t = tab[a - (lo >> 16):b - (lo >> 16) + 1] + np.uint64(self.before) if b >= a else np.zeros(0, np.uint64)
        sub = None
        if self.fmt == "u8s":
            a, b = (lo >> 8) + (1 if lo & 0xFF else 0), (hi - 1) >> 8
            sub = out[2][a - (lo >> 8):b - (lo >> 8) + 1] + np.uint16(self.before & 0xFFFF) if b >= a else \
                np.zeros(0, np.uint16)
        self.before += len(low)
        return low, t, sub


def line_index_pieces(co, begin: int = 0, end: Optional[int] = None, delim: int = 10, fmt: str = "u8s",
                      piece_bytes: int = 512 << 20, max_devices: Optional[int] = None, merge=None):
    """The u8s / u16b newline index of object bytes [begin, end) as it is produced: yields, in object order, each
    piece's (low, table slice, sub slice) of the whole range's tables (``PieceMerge``), so a caller can store
    piece k while later pieces are still being fetched and scanned (the streamed index PUT, verdict r5 #4).

    Pieces of at most ``piece_bytes`` (at least one per device entry) go round-robin to the device entries; each
    entry's persistent worker runs its pieces in order on rotating contexts, fetching piece k + 1 while piece k is
    scanned and read back (``_delim_piece_run``).  (Two workers per GPU fetching side by side were slower: 41 against ~50 GiB/s of
    GETs + H2D for a 4 GiB CSV, ``profiles/r06/e2e/``.)"""
    if fmt not in ("u8s", "u16b"):
        raise ValueError(f"streamed newline index forms: u8s or u16b, not {fmt!r}")
    end = co.size if end is None else end
    merge = merge or PieceMerge(begin, end, fmt)
    if end <= begin:
        return
    devs = devices(max_devices, co)
    n = len(devs)
    bounds = line_parts(begin, end, n, piece_bytes)
    futs = [cf.Future() for _ in bounds]
    stop = threading.Event()
    runs = []
    for e in range(min(n, len(bounds))):            # device entry e: pieces e, e + n, ... on its worker, in order
        jobs = [(bounds[k][0], bounds[k][1], futs[k]) for k in range(e, len(bounds), n)]
        runs.append(group_worker(devs[e], e).submit(_delim_piece_run, devs[e], co, jobs, delim, fmt, stop))
    try:
        for (lo, hi), f in zip(bounds, futs):
            yield merge.piece(lo, hi, f.result())
    finally:
        stop.set()                                  # (an abandoned or failed stream) the workers stop at their next piece
        cf.wait(runs)


_PIECE_CTXS = 3               # contexts a streamed-index worker rotates: fetch, scan, read-back in flight at once
# ranged-GET part of a streamed piece: 32 MiB (8 MiB parts let a piece's H2D start sooner in memory, 99 vs ~105 ms per
# 4 GiB, but over HTTP every GET is a request of its own: 12 vs 20 GiB/s, profiles/r06/e2e/timeline_8mib_parts.log)
_PIECE_GET_PART = _GET_PART


def _delim_piece_run(dev: int, co, jobs, delim: int, fmt: str, stop: threading.Event) -> None:
    """One device entry's pieces in order on its worker.  Three contexts of the worker rotate (their own streams,
    pinned staging and HBM buffers): piece k is fetched and its scan launched on one while a read-back thread collects
    piece k - 1 from another, so the worker's next GETs never wait for a read-back (whose D2H may queue behind the
    H2D copies of piece k on the same copy engine); piece k + 1's GETs are queued behind piece k's on one GET pool,
    so the GET stream does not drain at piece boundaries.  Each piece's (low, table[, sub]) is set on its future;
    the first failure on every remaining one."""
    ctxs = [get_context(dev, k) for k in range(_PIECE_CTXS)]
    mode = 4 if fmt == "u8s" else 3

    def launch(ctx, lo, hi, dp):
        rg = np.asarray([lo, hi], np.uint64)
        # capacity: 1 per 16 bytes for u8s, 1 per 64 for u16b (what "auto" stores below 1 per 128); a denser piece
        # is scanned again, sized, at its read-back
        cap = (hi - lo) // (16 if mode == 4 else 64) + 1024
        nbytes = ScanContext.out_bytes(cap, mode, rg)
        out = ctx.workspace("out", nbytes)
        ctx.delim_ranges_async(dp, hi - lo, lo, rg, delim, 1, 0, 0, out.ptr, mode, cap)
        # the whole output region read back right behind the scan (the entries' count is not known yet): in the
        # copy queue ahead of the next pieces' H2D copies, where a read-back issued after the count would wait
        hb = ctx.pinned("readback", nbytes)
        ctx.d2h_async(hb.ptr, out.ptr, nbytes)
        return ctx, rg, cap, out, dp, hb

    def collect(p, fut):
        ctx, rg, cap, out, dp, hb = p
        lo, hi = int(rg[0]), int(rg[1])
        try:
            try:
                cnt = ctx.delim_ranges_result(1)[0]
            except DPCapacityError:                  # denser than the capacity: again, synchronously, sized
                ctx.sync()
                r = ctx.delim_ranges(dp, hi - lo, lo, [(lo, hi)], delim=delim, out_mode=mode)
                fut.set_result((r[0], r[3], r[4]) if mode == 4 else (r[0], r[3]))
                return
            ctx.sync()                               # the read-back has landed
            a = hb.array
            low = a[:cnt * (1 if mode == 4 else 2)].view(np.uint8 if mode == 4 else np.uint16).copy()
            j0, nt = ScanContext.block_table_size(rg)
            t0 = ScanContext._tab_off(cap, mode)
            tab = a[t0:t0 + 8 * nt].view(np.uint64).copy()
            if lo & 0xFFFF:
                tab[0] = 0                           # the boundary below the first byte (ScanContext.block_table)
            if mode == 3:
                fut.set_result((low, tab))
                return
            s0, ns = ScanContext.sub_table_size(rg)
            u0 = ScanContext._sub_off(cap, rg)
            sub = a[u0:u0 + 2 * ns].view(np.uint16).copy()
            if lo & 0xFF:
                sub[0] = 0
            fut.set_result((low, tab, sub))
        except BaseException as e:
            fut.set_exception(e)
            raise
    reads = []
    pool = ctxs[0].get_pool(_GET_THREADS)         # one GET stream for every piece of the worker
    nxt = None                                      # the next piece's GETs, queued behind the current piece's

    def queue_gets(i):
        lo, hi, _ = jobs[i]
        if i >= _PIECE_CTXS:
            reads[i - _PIECE_CTXS].result()         # its context's previous piece is read back: staging is free
        host = ctxs[i % _PIECE_CTXS].pinned("object", hi - lo)
        return submit_gets(pool, co.storage, co.path.bucket, co.path.key, lo, hi, host, _PIECE_GET_PART)
    with cf.ThreadPoolExecutor(1, thread_name_prefix=f"dpscan-readback{dev}") as rb:
        try:
            for i, (lo, hi, fut) in enumerate(jobs):
                if stop.is_set():
                    raise RuntimeError("newline index stream abandoned")
                ctx = ctxs[i % _PIECE_CTXS]
                gets = nxt if nxt is not None else queue_gets(i)
                nxt = queue_gets(i + 1) if i + 1 < len(jobs) else None
                d = ctx.workspace("input", hi - lo + 64, placed=True)
                dp = d.ptr + (lo & 15)               # object offset and device address congruent mod 16
                land_gets(ctx, gets, dp)
                reads.append(rb.submit(collect, launch(ctx, lo, hi, dp), fut))
            cf.wait(reads)
        except BaseException as e:
            if nxt is not None:
                cancel_gets(nxt)
            cf.wait(reads)
            for _, _, fut in jobs:
                if not fut.done():
                    fut.set_exception(e)


def record_index_bytes(data, delim: int = 10, every_k: int = 1, emit_add: int = 0, device: int = 0,
                       u64: bool = True):
    """(offsets, number of delimiters) over host bytes already in memory (e.g. an inflated FASTQ stream)."""
    ctx = get_context(device)
    n = len(data)
    if n == 0:
        return np.zeros(0, np.uint64 if u64 else np.uint32), 0
    host = ctx.pinned("object", n)
    host.array[:n] = np.frombuffer(memoryview(data).cast("B"), np.uint8)
    d = ctx.workspace("input", n + 64, placed=True)
    ctx.h2d_async(d.ptr, host.ptr, n)
    return ctx.delim_index(d.ptr, n, 0, 0, n, delim=delim, every_k=every_k, emit_add=emit_add, u64=u64)
