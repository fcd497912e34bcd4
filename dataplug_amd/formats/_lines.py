"""Newline index artefact shared by the CSV and VCF plugins, and the slice boundaries derived from it.

The reference finds CSV/VCF slice boundaries at ``get()`` time by scanning a padded byte range in Python
(csv.py:52-105, vcf.py:88-149).  Here ``preprocess`` builds the sorted offsets of every ``'\\n'`` on the GPU
once — by default as uint8 low bytes plus the 16-bit entry counts before every 256-byte boundary and the
entry count below each 64 KiB boundary (u8s: the GPU writes about an eighth of the bytes of a uint64 index; the
counts and the block table are separate small objects) — stores them at ``s3://<bucket>.meta/<key>.lines``,
and a partition strategy resolves each
slice's exact byte range from that index, reproducing the reference's ``get()`` output (SURVEY.md §8(a)
formulas, restated below with the clamps the reference's buffer arithmetic implies).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import threading
from collections import OrderedDict
from typing import Optional, Tuple

import numpy as np

from ..storage.errors import ClientError
from ..version import __version__

LINES_SUFFIX = ".lines"
_PRELOAD_BYTES = 256 << 20
_BLOCK = 8192                      # entries per cached block for large indexes


_POOL = None
_POOL_PID = None
_PUT_THREADS = 3
_POOL_LOCK = threading.Lock()


def _put_pool() -> cf.ThreadPoolExecutor:
    """The persistent threads of an index's side and part PUTs (thread-local HTTP connections kept across calls).
    A forked child inherits the executor but not its threads, so a new one is made whenever the pid changes."""
    global _POOL, _POOL_PID
    with _POOL_LOCK:
        if _POOL is None or _POOL_PID != os.getpid():
            _POOL = cf.ThreadPoolExecutor(_PUT_THREADS, thread_name_prefix="dp-index-put")
            _POOL_PID = os.getpid()
        return _POOL


def _reset_pool_in_child():
    global _POOL, _POOL_PID, _POOL_LOCK
    _POOL, _POOL_PID, _POOL_LOCK = None, None, threading.Lock()


if hasattr(os, "register_at_fork"):
    os.register_at_fork(after_in_child=_reset_pool_in_child)


def store_line_index(cloud_object, offsets) -> dict:
    """PUT the index at ``<key>.lines``; returns the attributes that describe it.

    * ``scan.objects.ByteOffsets`` (``line_index_dtype="u8s"``): uint8 low bytes, the 256-byte counts (uint16 LE) at
      ``<key>.lines.sub`` and the 64 KiB block table (uint64 LE) at ``<key>.lines.blocks``, their first boundaries in
      the attributes;
    * ``scan.objects.BlockedOffsets`` (``line_index_dtype="u16b"``): uint16 LE low words,
      the 64 KiB block table (uint64 LE) at ``<key>.lines.blocks``, its first block in the attributes;
    * ``scan.objects.PagedOffsets`` (``"u32p"``): uint32 LE low words, the 4 GiB page counts in the attributes;
    * a plain array: uint64 LE."""
    key = cloud_object.meta_path.key + LINES_SUFFIX
    st, bucket = cloud_object.storage, cloud_object.meta_path.bucket
    meta = {"dataplug": __version__}
    attrs = {"line_index_key": key, "num_lines": int(len(offsets))}
    if hasattr(offsets, "sub"):
        skey, bkey = key + ".sub", key + ".blocks"
        # the counts and the table go up beside the low bytes (two requests in flight over HTTP)
        side = _put_pool().submit(lambda: [
            st.put_object(Body=np.ascontiguousarray(offsets.sub, "<u2").data, Bucket=bucket, Key=skey, Metadata=meta),
            st.put_object(Body=np.ascontiguousarray(offsets.table, "<u8").data, Bucket=bucket, Key=bkey,
                          Metadata=meta)])
        try:
            st.put_object(Body=np.ascontiguousarray(offsets.low, np.uint8).data, Bucket=bucket, Key=key, Metadata=meta)
        except BaseException:
            side.exception()                  # let the side PUTs finish; the low bytes' error is the one raised
            raise
        side.result()
        attrs.update(line_index_dtype="u8s", line_index_sub_key=skey, line_index_sub0=int(offsets.s0),
                     line_index_blocks_key=bkey, line_index_block0=int(offsets.j0))
    elif hasattr(offsets, "table"):
        st.put_object(Body=np.ascontiguousarray(offsets.low, "<u2").tobytes(), Bucket=bucket, Key=key, Metadata=meta)
        bkey = key + ".blocks"
        st.put_object(Body=np.ascontiguousarray(offsets.table, "<u8").tobytes(), Bucket=bucket, Key=bkey,
                      Metadata=meta)
        attrs.update(line_index_dtype="u16b", line_index_blocks_key=bkey, line_index_block0=int(offsets.j0))
    elif hasattr(offsets, "pages"):
        st.put_object(Body=np.ascontiguousarray(offsets.low, "<u4").tobytes(), Bucket=bucket, Key=key, Metadata=meta)
        attrs.update(line_index_dtype="u32p", line_index_pages=[int(x) for x in offsets.pages])
    else:
        st.put_object(Body=np.ascontiguousarray(offsets, "<u8").tobytes(), Bucket=bucket, Key=key, Metadata=meta)
    return attrs


# streamed index: least bytes per multipart part (S3's minimum is 5 MiB).  A piece's low bytes (~15 MB per 512 MiB of
# CSV) then go up as a part of their own, by reference: no concatenation on the consuming thread (16 MiB parts
# joined two pieces, ~3 ms of copying under the GIL each, profiles/r06/e2e/)
PART_MIN = 8 << 20


class MultipartWriter:
    """Byte arrays appended in order to one object, uploaded while later ones are still being produced: parts of at
    least ``part_min`` bytes go up as a multipart upload from the PUT threads as they fill; an object smaller than
    one part is one ``put_object`` at ``close``.  ``abort`` (or an exception in ``close``) removes the upload."""

    def __init__(self, storage, bucket: str, key: str, meta: dict, part_min: Optional[int] = None):
        self.st, self.bucket, self.key, self.meta = storage, bucket, key, meta
        self.part_min = PART_MIN if part_min is None else part_min
        self.pending, self.npend, self.size = [], 0, 0
        self.uid, self.futs = None, []

    def append(self, arr) -> None:
        a = np.ascontiguousarray(arr).reshape(-1).view(np.uint8)
        if a.nbytes:
            self.pending.append(a)
            self.npend += a.nbytes
            self.size += a.nbytes
        if self.npend >= self.part_min:
            self._flush()

    def _flush(self) -> None:
        data = self.pending[0] if len(self.pending) == 1 else np.concatenate(self.pending)
        self.pending, self.npend = [], 0
        if self.uid is None:
            self.uid = self.st.create_multipart_upload(Bucket=self.bucket, Key=self.key, Metadata=self.meta)["UploadId"]
        n = len(self.futs) + 1
        self.futs.append(_put_pool().submit(self.st.upload_part, Bucket=self.bucket, Key=self.key, PartNumber=n,
                                            UploadId=self.uid, Body=data.data))

    def close(self) -> int:
        """Finish the object (waits for its parts); returns its size."""
        if self.uid is None:
            data = np.concatenate(self.pending) if len(self.pending) > 1 else \
                (self.pending[0] if self.pending else np.zeros(0, np.uint8))
            self.st.put_object(Body=data.data, Bucket=self.bucket, Key=self.key, Metadata=self.meta)
            return self.size
        try:
            if self.npend:                        # the rest, in up to _PUT_THREADS parts uploaded side by side
                rest = np.concatenate(self.pending) if len(self.pending) > 1 else self.pending[0]
                step = max(5 << 20, -(-len(rest) // _PUT_THREADS))
                for a in range(0, len(rest), step):
                    self.pending, self.npend = [rest[a:a + step]], min(step, len(rest) - a)
                    self._flush()
            for f in self.futs:
                f.result()
            self.st.complete_multipart_upload(Bucket=self.bucket, Key=self.key, UploadId=self.uid, MultipartUpload={
                "Parts": [{"PartNumber": i + 1, "ETag": f.result()["ETag"]} for i, f in enumerate(self.futs)]})
        except BaseException:
            self.abort()
            raise
        self.uid = None                           # completed: nothing left to abort
        return self.size

    def abort(self) -> None:
        cf.wait(self.futs)
        if self.uid is not None:
            try:
                self.st.abort_multipart_upload(Bucket=self.bucket, Key=self.key, UploadId=self.uid)
            except ClientError:
                pass
            self.uid = None


def store_line_index_stream(cloud_object, pieces, fmt: str, merge) -> dict:
    """``store_line_index`` for an index produced piece by piece (``scan.objects.line_index_pieces``): the low
    bytes / words and the 256-byte counts go up as multipart uploads while later pieces are still being fetched and
    scanned; the block table (8 B per 64 KiB) is PUT at the end.  Stores the same objects and returns the same
    attributes as ``store_line_index`` of the merged index."""
    key = cloud_object.meta_path.key + LINES_SUFFIX
    st, bucket = cloud_object.storage, cloud_object.meta_path.bucket
    meta = {"dataplug": __version__}
    skey, bkey = key + ".sub", key + ".blocks"
    low_w = MultipartWriter(st, bucket, key, meta)
    sub_w = MultipartWriter(st, bucket, skey, meta) if fmt == "u8s" else None
    tabs = [merge.head_table()]
    if sub_w is not None:
        sub_w.append(merge.head_sub().astype("<u2"))
    try:
        for low, tab, sub in pieces:
            low_w.append(low.astype(np.uint8 if fmt == "u8s" else "<u2", copy=False))
            if sub_w is not None:
                sub_w.append(sub.astype("<u2", copy=False))
            tabs.append(tab)
        count = low_w.close() // (1 if fmt == "u8s" else 2)
        if sub_w is not None:
            sub_w.close()
    except BaseException:
        low_w.abort()
        if sub_w is not None:
            sub_w.abort()
        raise
    st.put_object(Body=np.ascontiguousarray(np.concatenate(tabs), "<u8").data, Bucket=bucket, Key=bkey, Metadata=meta)
    attrs = {"line_index_key": key, "num_lines": int(count), "line_index_dtype": fmt, "line_index_blocks_key": bkey,
             "line_index_block0": int(merge.J0)}
    if fmt == "u8s":
        attrs.update(line_index_sub_key=skey, line_index_sub0=int(merge.S0))
    return attrs


STREAM_PIECE = 512 << 20           # streamed index: object bytes per scanned piece


def index_object(cloud_object, begin: int = 0, index_format: str = "auto", piece_bytes: int = STREAM_PIECE) -> dict:
    """Build the newline index of object bytes [begin, size) on the GPUs and store it; returns its attributes.
    ``index_format`` "auto" takes u8s or u16b by the object's newline density (``scan.objects.line_index_form``).
    A u8s / u16b index of more than one piece is stored as it is produced (``store_line_index_stream``: the PUTs
    overlap the later pieces' GETs, H2D copies and scans); other forms and single pieces are built, then stored."""
    from ..scan import objects as so
    end = cloud_object.size
    fmt = so.line_index_form(cloud_object, begin, end) if index_format == "auto" else index_format
    if fmt in ("u8s", "u16b") and end - begin > piece_bytes:
        merge = so.PieceMerge(begin, end, fmt)
        pieces = so.line_index_pieces(cloud_object, begin, end, fmt=fmt, piece_bytes=piece_bytes, merge=merge)
        try:
            return store_line_index_stream(cloud_object, pieces, fmt, merge)
        finally:
            pieces.close()
    return store_line_index(cloud_object, so.line_index_object(cloud_object, begin=begin, end=end, fmt=fmt))


class LineIndex:
    """Sorted newline offsets; ``nxt(x)`` = 1 + first '\n' at or after x (None if none).

    Reads every stored form (uint64 words; uint32 low words + 4 GiB page counts; uint16 low words + 64 KiB
    block table; uint8 low bytes + 256-byte counts + 64 KiB block table), fetching blocks of entries by ranged GETs
    when the index is large (for the uint8 form with the 256-byte counts of the blocks they span)."""

    def __init__(self, offsets: Optional[np.ndarray] = None, storage=None, bucket: str = "", key: str = "",
                 count: Optional[int] = None, pages: Optional[list] = None, blocks: Optional[np.ndarray] = None,
                 block0: int = 0, sub_key: Optional[str] = None, sub0: int = 0):
        self._arr = None if offsets is None else np.asarray(offsets, dtype=np.uint64)
        self._storage, self._bucket, self._key = storage, bucket, key
        self._pages = None if pages is None else np.asarray(pages, np.int64)
        self._blocks_tab = None if blocks is None else np.asarray(blocks, np.uint64)   # converted once
        self._block0 = int(block0)
        self._sub_key, self._sub0 = sub_key, int(sub0)
        self._item = 1 if sub_key is not None else (2 if blocks is not None else (4 if pages is not None else 8))
        self._blocks: "OrderedDict[int, np.ndarray]" = OrderedDict()
        if self._arr is None:
            if count is None:
                count = int(storage.head_object(Bucket=bucket, Key=key)["ContentLength"]) // self._item
            self.count = int(count)
            # a preload of the uint8 form also reads every 256-byte count (2 B per 256 object bytes, whatever the
            # number of entries): a sparse index of a large object is read block by block instead
            side = 2 * 256 * len(self._blocks_tab) if self._item == 1 else 0
            if self.count * self._item + side <= _PRELOAD_BYTES:
                self._arr = self._fetch(0, self.count)
        else:
            self.count = len(self._arr)

    @classmethod
    def of(cls, cloud_object) -> "LineIndex":
        attrs = cloud_object.attributes
        key = getattr(attrs, "line_index_key", None) if attrs is not None else None
        if not key:
            raise KeyError(f"{cloud_object!r} has no newline index: preprocess it with dataplug_amd (line_index=True)")
        dt = getattr(attrs, "line_index_dtype", None)
        kw = {}
        if dt == "u32p":
            kw["pages"] = list(getattr(attrs, "line_index_pages"))
        elif dt in ("u16b", "u8s"):
            res = cloud_object.storage.get_object(Bucket=cloud_object.meta_path.bucket,
                                                  Key=getattr(attrs, "line_index_blocks_key"))
            kw["blocks"] = np.frombuffer(res["Body"].read(), "<u8")
            kw["block0"] = int(getattr(attrs, "line_index_block0"))
            if dt == "u8s":
                kw["sub_key"] = getattr(attrs, "line_index_sub_key")
                kw["sub0"] = int(getattr(attrs, "line_index_sub0"))
        return cls(storage=cloud_object.storage, bucket=cloud_object.meta_path.bucket, key=key,
                   count=getattr(attrs, "num_lines", None), **kw)

    def _fetch(self, i0: int, i1: int) -> np.ndarray:
        if i1 <= i0:
            return np.zeros(0, np.uint64)
        it = self._item
        res = self._storage.get_object(Bucket=self._bucket, Key=self._key, Range=f"bytes={it * i0}-{it * i1 - 1}")
        raw = res["Body"].read()
        if it == 8:
            return np.frombuffer(raw, dtype="<u8").astype(np.uint64, copy=False)
        idx = np.arange(i0, i1, dtype=np.int64)
        if it == 4:
            page = np.searchsorted(self._pages, idx, side="right").astype(np.uint64)
            return (page << np.uint64(32)) | np.frombuffer(raw, dtype="<u4").astype(np.uint64)
        if it == 1:
            return self._decode_bytes(idx, np.frombuffer(raw, dtype=np.uint8))
        blk = np.searchsorted(self._blocks_tab, idx, side="right").astype(np.uint64) - np.uint64(1)
        return ((blk + np.uint64(self._block0)) << np.uint64(16)) | np.frombuffer(raw, dtype="<u2").astype(np.uint64)

    _SUB_GAP = 4                      # needed 64 KiB blocks at most this many apart share one ranged GET of counts

    def _decode_bytes(self, idx: np.ndarray, low: np.ndarray) -> np.ndarray:
        """Offsets of entries ``idx`` (ascending) of the uint8 form from their low bytes: the 256-byte counts are
        read only for the 64 KiB blocks the entries lie in (runs of nearby blocks coalesced into one GET), so the
        bytes read follow the entries, not the object bytes they span."""
        from ..scan.objects import sub_counts
        tab, s0, j0 = self._blocks_tab, self._sub0, self._block0
        blk = np.searchsorted(tab, idx.astype(np.uint64), side="right").astype(np.int64) - 1
        need = np.unique(blk)
        cut = np.flatnonzero(np.diff(need) > self._SUB_GAP) + 1
        s = np.empty(len(idx), np.uint64)
        for run in np.split(need, cut):
            ja, jb = int(run[0]), int(run[-1])
            sa = max(0, ((j0 + ja) << 8) - s0)
            sb = ((j0 + jb + 1) << 8) - s0
            res = self._storage.get_object(Bucket=self._bucket, Key=self._sub_key, Range=f"bytes={2 * sa}-{2 * sb - 1}")
            c = sub_counts(np.frombuffer(res["Body"].read(), dtype="<u2"), tab, s0, j0, sa)
            a, b = np.searchsorted(blk, [ja, jb + 1])
            s[a:b] = (np.searchsorted(c, idx[a:b].astype(np.uint64), side="right").astype(np.int64) + (sa - 1)).astype(np.uint64)
        return ((s + np.uint64(s0)) << np.uint64(8)) | low.astype(np.uint64)

    def _block(self, b: int) -> np.ndarray:
        blk = self._blocks.get(b)
        if blk is None:
            blk = self._fetch(b * _BLOCK, min(self.count, (b + 1) * _BLOCK))
            self._blocks[b] = blk
            if len(self._blocks) > 64:
                self._blocks.popitem(last=False)
        return blk

    def _search(self, x: int) -> int:
        """Index of the first entry >= x (``count`` if none)."""
        if self._arr is not None:
            return int(np.searchsorted(self._arr, np.uint64(x)))
        nb = -(-self.count // _BLOCK)
        lo, hi = 0, nb                      # first block whose last entry >= x
        while lo < hi:
            mid = (lo + hi) // 2
            last = self._block(mid)[-1]
            if int(last) >= x:
                hi = mid
            else:
                lo = mid + 1
        if lo == nb:
            return self.count
        return lo * _BLOCK + int(np.searchsorted(self._block(lo), np.uint64(x)))

    def value(self, i: int) -> int:
        if self._arr is not None:
            return int(self._arr[i])
        return int(self._block(i // _BLOCK)[i % _BLOCK])

    def nxt(self, x: int) -> Optional[int]:
        i = self._search(x)
        return self.value(i) + 1 if i < self.count else None

    def contains(self, x: int) -> bool:
        i = self._search(x)
        return i < self.count and self.value(i) == x


class SliceError(ValueError):
    """The reference's ``get()`` fails for this slice (kept as an error, not papered over).  A ``ValueError``:
    what the reference raises for the negative ``seek`` of csv.py:75."""


class SliceRangeError(ClientError, SliceError):
    """The reference's ``get()`` ends in a ranged GET that starts past the end of the object, which S3 answers
    with InvalidRange (HTTP 416), a botocore ``ClientError``: its CSV buffer expansion (csv.py:81-94) writes
    each fetched range after the read position and never reads it, so it fetches further and further on until
    that happens; its VCF expansion (vcf.py:117-136) does when no '\\n' follows before the end.  Raised as the
    storage ``ClientError`` the reference's caller would see (and, as every ``SliceError``, a ``ValueError``);
    pinned by the golden slices of rows longer than the padding (tests/golden/csv_slices.json ``wide_csv``)."""

    def __init__(self, message: str):
        self.detail = message
        ClientError.__init__(self, "InvalidRange", "GetObject", message, 416)

    def __reduce__(self):                 # slices travel to joblib workers
        return (SliceRangeError, (self.detail,))


def slice_error(e: SliceError) -> SliceError:
    """A fresh exception of the same kind (a slice raises it at every get())."""
    return SliceRangeError(e.detail) if isinstance(e, SliceRangeError) else SliceError(*e.args)


def csv_body(lines: LineIndex, size: int, r0: int, r1: int, chunk_id: int, num_chunks: int,
             padding: int) -> Tuple[int, int]:
    """Object bytes [start, end) that ``CSVSlice.get`` (csv.py:52-105) returns (after the header prefix).

    The reference reads ``bytes=r0-r1`` (inclusive) → buffer end ``be = min(r1 + 1, size)``.
    * start: chunk 0 → r0; else r0 itself when byte r0 is '\\n' (that line is then in two slices), otherwise
      1 + the first '\\n' after r0, capped at ``be`` (readline stops at the buffer end).
    * end: last chunk → ``be``; otherwise 1 + the first '\\n' at or after ``be - padding - 1``.  The
      reference seeks to a negative position when ``be - r0 <= padding`` (ValueError), and its buffer-
      expansion loop never finds a '\\n' it did not already hold, so a missing '\\n' in
      [be - padding - 1, be) is an error as well."""
    be = min(r1 + 1, size)
    if chunk_id == 0:
        start = r0
    elif lines.contains(r0):
        start = r0
    else:
        n = lines.nxt(r0 + 1)
        start = be if n is None else min(n, be)
    if chunk_id == num_chunks - 1:
        return start, be
    if be - r0 <= padding:
        raise SliceError(f"slice {chunk_id} holds {be - r0} bytes <= padding {padding}: the reference's "
                         f"CSVSlice.get seeks to a negative position (ValueError)")
    n = lines.nxt(be - padding - 1)
    if n is None or n > be:
        raise SliceRangeError(f"slice {chunk_id}: no newline in the last {padding + 1} bytes of its range; the "
                              f"reference's buffer expansion (csv.py:81-94) fetches ranges until one starts past "
                              f"the end of the object")
    return start, n


def vcf_body(lines: LineIndex, size: int, r0: int, r1: int, chunk_id: int, num_chunks: int) -> Tuple[int, int]:
    """Object bytes [start, end) of a ``VCFSlice.get`` body (vcf.py:88-149).

    Buffer end ``be = min(r1 + 1, size)``.  start: chunk 0 → r0 (= body_offset); else 1 + the first '\\n' at
    or after r0, capped at ``be``.  end: last chunk → ``be``; else 1 + the first '\\n' at or after ``be - 1``
    (the reference's expansion reads further ranges until it sees one; none before EOF → its GET past the
    end fails)."""
    be = min(r1 + 1, size)
    if chunk_id == 0:
        start = r0
    else:
        n = lines.nxt(r0)
        start = be if n is None else min(n, be)
    if chunk_id == num_chunks - 1:
        return start, be
    n = lines.nxt(be - 1)
    if n is None:
        raise SliceRangeError(f"slice {chunk_id}: no newline after byte {be - 1}; the reference's range "
                              f"expansion requests bytes past the end of the object")
    return start, n
