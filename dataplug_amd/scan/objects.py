"""Object-level index builds: storage → pinned host → HBM → HIP scan → host index.

These are what the format plugins call.  Everything computational runs in libdpscan (HIP); the host side
only moves bytes and stitches per-GPU results in chunk order.  Multi-GPU: an object's map chunks are
independent (preprocess.py:39-51 of the reference), so the chunk list is cut into contiguous groups, one
per GPU, each scanned by one launch on its own device; no collective.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ._lib import DPScanUnavailable
from ..dist import split_groups
from ..storage.ranges import GET_PART as _GET_PART, GET_THREADS as _GET_THREADS, read_range_into
from .device import ScanContext, device_count, get_context

_HALO0 = 64 << 10             # first look-ahead window when a header line crosses the fetched bytes
# bytes one FASTA launch holds in HBM at most: a GPU's chunk group larger than this (an object far beyond
# 288 GB x GPUs, or a small budget set for tests) is scanned in several passes of whole chunks
MAX_LAUNCH_BYTES = 64 << 30


def max_launch_bytes() -> int:
    return int(os.environ.get("DATAPLUG_AMD_MAX_LAUNCH_BYTES", MAX_LAUNCH_BYTES))


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
                    part: Optional[int] = None, threads: int = _GET_THREADS):
    """Object bytes [lo, hi) into device memory at ``d_ptr``: parallel ranged GETs into the context's pinned
    staging buffer, each part's H2D copy issued on the context stream as soon as that part has landed, so
    the PCIe copy overlaps the remaining GETs (storage -> pinned -> HBM pipeline).
    Returns the pinned buffer (valid until the context's next fetch).  The copies are asynchronous: work
    enqueued afterwards on the same stream (the scan) sees the bytes."""
    n = hi - lo
    part = part or _GET_PART
    host = ctx.pinned("object", max(n, 1))
    if n <= 0:
        return host
    view = host.view(n)
    starts = list(range(0, n, part))
    if len(starts) == 1:
        read_range_into(storage, bucket, key, lo, hi, view, part=part, threads=threads)
        ctx.h2d_async(d_ptr, host.ptr, n)
        return host

    def one(a: int) -> int:
        read_range_into(storage, bucket, key, lo + a, lo + min(n, a + part), view[a:], part=part, threads=1)
        return a

    with cf.ThreadPoolExecutor(min(threads, len(starts))) as ex:
        futs = [ex.submit(one, a) for a in starts]
        for f in cf.as_completed(futs):       # H2D issued from this (the context's) thread only
            a = f.result()
            ctx.h2d_async(d_ptr + a, host.ptr + a, min(n, a + part) - a)
    return host


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


# ------------------------------------------------------------------------------------------ FASTA
@dataclass(frozen=True)
class FastaGroup:
    """One GPU's share of a FASTA chunk plan: chunks [i0, i1) of the plan (contiguous, so the outputs
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


def fasta_groups(plan: Sequence[Tuple[int, int]], n_groups: int, size: int, halo: int = _HALO0) -> List[FastaGroup]:
    """The multi-GPU split of one object's chunk plan (the reference runs the chunks as
    independent map jobs, preprocess.py:39-51): ``split_groups`` of the chunk list over ``n_groups`` GPUs.
    Used by ``fasta_index_object`` and by bench.py's multi-GPU line (one thread or rank per group)."""
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


def _fasta_group(dev: int, co, plan: Sequence[Tuple[int, int]], g: FastaGroup, u64: bool) -> np.ndarray:
    ctx = get_context(dev)
    size = co.size
    parts = []
    for p_ in fasta_passes(plan, g, size, max_launch_bytes()):
        n = p_.buf_hi - p_.lo
        d = ctx.workspace("input", n + 64)
        fetch_to_device(ctx, co.storage, co.path.bucket, co.path.key, p_.lo, p_.buf_hi, d.ptr)
        pairs, pending, _ = ctx.fasta_index(d.ptr, n, p_.lo, size, p_.chunks(plan), u64=u64)
        for p in pending[pending >= 0]:
            start = int(pairs[p, 0])
            end = resolve_line_end(ctx, co.storage, co.path.bucket, co.path.key, size, p_.buf_hi)
            if not u64 and end > 0xFFFFFFFF:
                raise OverflowError(f"FASTA offset {end} does not fit the uint32 index (header at {start})")
            pairs[p, 1] = end
        parts.append(pairs)
    return parts[0] if len(parts) == 1 else np.concatenate(parts)


def fasta_index_object(co, plan: Sequence[Tuple[int, int]], u64: bool = False,
                       max_devices: Optional[int] = None) -> np.ndarray:
    """(n, 2) (start, end) pairs of every chunk of ``plan`` concatenated in chunk order — the index
    ``merge_fasta_metadata`` (fasta.py:66-74) assembles from the per-chunk map outputs."""
    if not plan:
        return np.zeros((0, 2), np.uint64 if u64 else np.uint32)
    devs = devices(max_devices, co)
    groups = fasta_groups(plan, len(devs), co.size)
    if len(groups) == 1:
        return _fasta_group(devs[0], co, plan, groups[0], u64)
    with cf.ThreadPoolExecutor(len(groups)) as ex:
        futs = [ex.submit(_fasta_group, devs[k], co, plan, g, u64) for k, g in enumerate(groups)]
        parts = [f.result() for f in futs]
    return np.concatenate(parts)


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


INDEX_FORMATS = ("u16b", "u32p", "u64")


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
    d = ctx.workspace("input", n + 64)
    dp = d.ptr + (lo & 15)                # object offset and device address congruent mod 16 (out_mode 3 grid)
    fetch_to_device(ctx, co.storage, co.path.bucket, co.path.key, lo, hi, dp)
    if fmt == "u64":
        return ctx.delim_index(dp, n, lo, lo, hi, delim=delim, every_k=every_k, emit_add=emit_add, u64=True)
    if fmt == "u32p":
        rg = page_ranges(lo, hi)
        low, nd, ends = ctx.delim_ranges(dp, n, lo, rg, delim=delim, out_mode=2)
        return low, [(r, int(e)) for r, e in zip(rg, ends)]
    low, nd, ends, tab = ctx.delim_ranges(dp, n, lo, [(lo, hi)], delim=delim, out_mode=3)
    return low, tab


def line_index_object(co, begin: int = 0, end: Optional[int] = None, delim: int = 10,
                      max_devices: Optional[int] = None, part_bytes: int = 16 << 30, fmt: str = "u64"):
    """Sorted offsets of every ``delim`` byte of object bytes [begin, end) in one of ``INDEX_FORMATS``:
    ``u64`` a uint64 array; ``u32p`` a ``PagedOffsets`` (uint32 low words + 4 GiB page counts); ``u16b`` a
    ``BlockedOffsets`` (uint16 low words + a 64 KiB block table) — the GPU writes 8, 4 or 2 bytes per offset.

    The range is cut into independent parts (at most ``part_bytes`` each, at least one per GPU) scanned
    round-robin on the GPUs and concatenated in order."""
    if fmt not in INDEX_FORMATS:
        raise ValueError(f"index format must be one of {INDEX_FORMATS}, not {fmt!r}")
    end = co.size if end is None else end
    if end <= begin:
        return {"u64": np.zeros(0, np.uint64), "u32p": PagedOffsets(np.zeros(0, np.uint32), []),
                "u16b": BlockedOffsets(np.zeros(0, np.uint16), np.zeros(1, np.uint64), begin >> 16)}[fmt]
    devs = devices(max_devices, co)
    bounds = line_parts(begin, end, len(devs), part_bytes)

    def run(k: int):
        lo, hi = bounds[k]
        r = _delim_group(devs[k % len(devs)], co, lo, hi, delim, 1, 0, fmt=fmt)
        return r[0] if fmt == "u64" else r

    if len(bounds) == 1:
        out = [run(0)]
    else:
        # one worker per GPU; parts of the same GPU run in order on that GPU's thread
        by_dev = {}
        for k in range(len(bounds)):
            by_dev.setdefault(k % len(devs), []).append(k)
        out = [None] * len(bounds)

        def worker(ks):
            for k in ks:
                out[k] = run(k)

        with cf.ThreadPoolExecutor(len(by_dev)) as ex:
            list(ex.map(worker, by_dev.values()))
    if fmt == "u64":
        return np.concatenate(out)
    low = np.concatenate([o[0] for o in out])
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
    # u16b: table[j - J0] = offsets before j * 64 KiB; a boundary inside part k comes from part k's own table
    # (its count within the part) plus every earlier part's count
    J0, J1 = begin >> 16, (end - 1) >> 16
    table = np.zeros(J1 - J0 + 1, np.uint64)
    before = 0
    for (lo, hi), (lw, tab) in zip(bounds, out):
        j0 = lo >> 16
        js = np.arange(max(j0, J0), ((hi - 1) >> 16) + 1, dtype=np.int64)
        inside = (js << 16) >= lo                        # boundaries at or after the part's first byte
        table[js[inside] - J0] = np.uint64(before) + tab[js[inside] - j0]
        before += len(lw)
    return BlockedOffsets(low, table, J0)


def record_index_bytes(data, delim: int = 10, every_k: int = 1, emit_add: int = 0, device: int = 0,
                       u64: bool = True):
    """(offsets, number of delimiters) over host bytes already in memory (e.g. an inflated FASTQ stream)."""
    ctx = get_context(device)
    n = len(data)
    if n == 0:
        return np.zeros(0, np.uint64 if u64 else np.uint32), 0
    host = ctx.pinned("object", n)
    host.array[:n] = np.frombuffer(memoryview(data).cast("B"), np.uint8)
    d = ctx.workspace("input", n + 64)
    ctx.h2d_async(d.ptr, host.ptr, n)
    return ctx.delim_index(d.ptr, n, 0, 0, n, delim=delim, every_k=every_k, emit_add=emit_add, u64=u64)
