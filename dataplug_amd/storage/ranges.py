"""Ranged reads: parallel ranged GETs into caller memory, and coalesced reads of many small ranges.

Both are host-side plumbing of the storage → host path.  S3 ``Range`` headers
are inclusive (``bytes=a-b``); everything here takes half-open ``[lo, hi)`` object offsets.
"""
from __future__ import annotations

import concurrent.futures as cf
from typing import Dict, List, Sequence, Tuple

import numpy as np

GET_PART = 32 << 20          # ranged-GET part size for parallel fetches
GET_THREADS = 16
COALESCE_GAP = 1 << 20       # two wanted ranges closer than this are fetched by one GET


def read_range_into(storage, bucket: str, key: str, lo: int, hi: int, out: memoryview,
                    part: int = GET_PART, threads: int = GET_THREADS) -> None:
    """Object bytes [lo, hi) into ``out`` (len >= hi - lo) with parallel ranged GETs (inclusive Range)."""
    n = hi - lo
    if n <= 0:
        return
    out = out.cast("B") if out.format != "B" else out

    def one(a: int) -> None:
        b = min(n, a + part)
        res = storage.get_object(Bucket=bucket, Key=key, Range=f"bytes={lo + a}-{lo + b - 1}")
        body = res["Body"]
        got = a
        with body:
            while got < b:
                r = body.readinto(out[got:b])
                if not r:
                    raise IOError(f"short read of {bucket}/{key} at {lo + got}")
                got += r

    starts = list(range(0, n, part))
    if len(starts) == 1:
        one(0)
        return
    with cf.ThreadPoolExecutor(min(threads, len(starts))) as ex:
        list(ex.map(one, starts))


def coalesce(ranges: Sequence[Tuple[int, int]], gap: int = COALESCE_GAP) -> List[Tuple[int, int]]:
    """Sorted, merged extents covering every non-empty [lo, hi) of ``ranges``; extents closer than
    ``gap`` bytes are joined (one GET instead of two, at the price of at most ``gap`` unwanted bytes)."""
    rs = sorted((int(a), int(b)) for a, b in ranges if b > a)
    out: List[List[int]] = []
    for a, b in rs:
        if out and a <= out[-1][1] + gap:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return [(a, b) for a, b in out]


class Extents:
    """Object bytes of a set of coalesced extents, held in one host buffer; ``view(lo, hi)`` of any
    wanted range inside one extent."""

    def __init__(self, storage, bucket: str, key: str, ranges: Sequence[Tuple[int, int]],
                 gap: int = COALESCE_GAP, threads: int = GET_THREADS):
        self.extents = coalesce(ranges, gap)
        total = sum(b - a for a, b in self.extents)
        self.buf = np.empty(max(1, total), np.uint8)
        self._where: Dict[int, int] = {}
        self.starts = np.array([a for a, _ in self.extents], np.int64)
        off = 0
        jobs = []
        for a, b in self.extents:
            self._where[a] = off
            # split every extent into GET parts so that one large extent still fans out
            for p in range(a, b, GET_PART):
                q = min(b, p + GET_PART)
                jobs.append((p, q, off + (p - a)))
            off += b - a
        mv = memoryview(self.buf)

        def one(job):
            p, q, o = job
            read_range_into(storage, bucket, key, p, q, mv[o:o + (q - p)], threads=1)

        if len(jobs) == 1:
            one(jobs[0])
        elif jobs:
            with cf.ThreadPoolExecutor(min(threads, len(jobs))) as ex:
                for f in [ex.submit(one, j) for j in jobs]:
                    f.result()
        self.n_gets = len(jobs)

    def view(self, lo: int, hi: int) -> memoryview:
        i = int(np.searchsorted(self.starts, lo, side="right")) - 1
        if i < 0 or not (self.extents[i][0] <= lo and hi <= self.extents[i][1]):
            raise KeyError(f"[{lo}, {hi}) was not fetched")
        a = self.extents[i][0]
        o = self._where[a] + (lo - a)
        return memoryview(self.buf)[o:o + (hi - lo)]
