"""Streamed gzip line / read index: storage → host inflate (bounded pieces) → pinned → HBM → newline scan.

What gztool does for the reference's GZipText / FASTQGZip preprocess (dataplug/formats/compressed/
gzipped.py:46-153: the object streamed into ``gztool -i -x -I`` in 64 KiB writes, then ``-ell`` for the line
count and the window table), rebuilt as a pipeline whose host memory does not grow with the object:

* an inflater thread pulls compressed bytes from the GET body and inflates them (libdpgz) into one of a few
  pinned piece buffers of ``piece_bytes`` — a plain gzip stream on the thread pool by speculative deflate
  block starts (``dpgz_par``; zlib on one core when only one thread is available), BGZF-style members
  (compressed size in their header) on the thread pool, member by member straight to their place in the
  piece;
* the calling thread copies each finished piece to HBM and runs ``dp_delim_ranges`` on it with the newline
  ordinal carried from the previous pieces, so ``every_k = record_lines`` selects read ends across piece
  boundaries (FASTQ: every 4th '\\n' + 1), while the inflater fills the next piece;
* access points (libdpgz: deflate block boundaries every ``span`` inflated bytes, plus member starts) come
  with their 32 KiB windows and the byte before them; their line numbers follow from the carried newline
  count, the piece's read ends and a count over at most ``record_lines`` lines of the piece.

Host memory: ``n_pieces`` pinned pieces + one compressed read buffer + the spooled outputs' in-memory part
(``SPOOL_MEM`` each), independent of the object size.  Outputs: read ends (uint64, spooled), the windows
blob (spooled), the window-table rows, the line count.
"""
from __future__ import annotations

import os
import queue
import tempfile
import threading
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import numpy as np

from .. import gz as gzlib
from ._lib import DPCapacityError
from .device import ScanContext

PIECE_BYTES = 64 << 20
READ_BYTES = 1 << 20          # compressed bytes per GET-body read (the reference writes 64 KiB pieces)
BGZF_BATCH = 16 << 20         # compressed bytes scanned for complete BGZF members at a time
SPOOL_MEM = 64 << 20
PAR_READ_BYTES = 4 << 20      # compressed bytes per read while a plain stream is inflated in parallel


def pool_threads() -> int:
    """Inflate threads for member-parallel input: the CPUs this process may use, capped by the box's share
    (OMP_NUM_THREADS, 16 on the GPU box where os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, min(n, cap))


@dataclass
class _Piece:
    slot: int
    o0: int                              # inflated offset of the piece's first byte
    n: int
    points: np.ndarray                   # POINTEX_DTYPE rows with o0 <= out_byte <= o0 + n
    windows: bytes


@dataclass
class GzIndex:
    """What the pipeline produced (outputs spooled; rewind before reading)."""
    ends: "tempfile.SpooledTemporaryFile"          # uint64 LE read-end offsets (every record_lines-th '\\n' + 1)
    windows: "tempfile.SpooledTemporaryFile"       # 32 KiB windows of the access points, concatenated
    rows: List[list] = field(default_factory=list)  # window table rows (WINDOW_COLUMNS of gzipped.py)
    newlines: int = 0
    num_records: int = 0
    uncompressed_size: int = 0
    members: int = 0
    last_byte: int = -1
    bgzf: bool = False
    pieces: int = 0

    @property
    def total_lines(self) -> int:
        """Lines of the inflated stream: '\\n' count, +1 for a final unterminated line (gztool's own
        convention for that case is unpinned)."""
        return self.newlines + (1 if self.uncompressed_size and self.last_byte != 10 else 0)


class _Inflater(threading.Thread):
    """Fills pinned piece buffers from the compressed stream; hands finished pieces to the scan thread."""

    def __init__(self, read: Callable[[int], bytes], pieces: List[np.ndarray], span: int, threads: int,
                 region_bytes: Optional[int] = None):
        super().__init__(daemon=True, name="dpgz-inflate")
        self.read, self.pieces, self.span, self.threads = read, pieces, span, threads
        self.region_bytes = region_bytes
        self.free: "queue.Queue[int]" = queue.Queue()
        for i in range(len(pieces)):
            self.free.put(i)
        self.ready: "queue.Queue[Optional[_Piece]]" = queue.Queue()
        self.error: Optional[BaseException] = None
        self.bgzf = False
        self.members = 0
        self.stop = threading.Event()

    def run(self):
        try:
            first = self.read(READ_BYTES)
            if gzlib.is_bgzf(first):
                self.bgzf = True
                self._run_bgzf(first)
            elif self.threads > 1:
                self._run_parallel(first)
            else:
                self._run_stream(first)
        except BaseException as e:                      # surfaced by the scan thread
            self.error = e
        finally:
            self.ready.put(None)

    def _take_slot(self) -> Optional[int]:
        while not self.stop.is_set():
            try:
                return self.free.get(timeout=0.5)
            except queue.Empty:
                continue
        return None

    def _run_stream(self, first: bytes):
        st = gzlib.InflateStream(self.span)
        try:
            buf, pos, final = first, 0, len(first) == 0
            o0 = 0
            while True:
                slot = self._take_slot()
                if slot is None:
                    return
                out = self.pieces[slot]
                filled, end = 0, False
                while filled < len(out):
                    if pos == len(buf) and not final:
                        buf, pos = self.read(READ_BYTES), 0
                        final = len(buf) == 0
                    c, p, end = st.inflate(memoryview(buf)[pos:], final, out, filled, len(out) - filled)
                    pos += c
                    filled += p
                    if end:
                        break
                pts, win = st.take()
                self.members = st.state()[2]
                self.ready.put(_Piece(slot, o0, filled, pts, win))
                o0 += filled
                if end:
                    return
        finally:
            st.close()

    def _run_parallel(self, first: bytes):
        """A plain gzip stream inflated on the thread pool (libdpgz dpgz_par_*: speculative block starts,
        marker windows, CRC-checked), drained into the pieces in order."""
        pi = gzlib.ParInflate(self.span, self.threads, region_bytes=self.region_bytes)
        # compressed bytes are read ahead on their own thread (up to 16 reads), so the GET body's copies
        # overlap the engine's batches
        inq: "queue.Queue[Optional[bytes]]" = queue.Queue(maxsize=16)
        stop_reading = threading.Event()

        def reader():
            try:
                while not stop_reading.is_set():
                    data = self.read(PAR_READ_BYTES)
                    while not stop_reading.is_set():
                        try:
                            inq.put(data, timeout=0.5)
                            break
                        except queue.Full:
                            continue
                    if not data:
                        return
            except BaseException as e:                   # surfaced by the inflater loop
                self.error = e
                while not stop_reading.is_set():         # wake the consumer unless it has already left
                    try:
                        inq.put(b"", timeout=0.5)
                        break
                    except queue.Full:
                        continue

        rt = threading.Thread(target=reader, daemon=True, name="dpgz-read")
        try:
            final = len(first) == 0
            if not final:
                rt.start()
            pi.feed(first, final)
            o0, slot, filled, out = 0, None, 0, None
            while True:
                while True:                                # move the inflated bytes into pieces
                    if slot is None:
                        slot = self._take_slot()
                        if slot is None:
                            return
                        out, filled = self.pieces[slot], 0
                    n = pi.read_into(out, filled, len(out) - filled)
                    filled += n
                    if filled == len(out):
                        pts, win = pi.take(o0 + filled)
                        self.ready.put(_Piece(slot, o0, filled, pts, win))
                        o0 += filled
                        slot = None
                        continue
                    if n == 0:
                        break
                st = pi.stats()
                self.members = st["members"]
                if st["ended"]:
                    if slot is None:
                        slot = self._take_slot()
                        if slot is None:
                            return
                        filled = 0
                    pts, win = pi.take(o0 + filled)
                    self.ready.put(_Piece(slot, o0, filled, pts, win))
                    return
                if final:
                    raise ValueError("gzip stream: truncated")
                data = inq.get()
                if self.error is not None:
                    raise self.error
                final = len(data) == 0
                pi.feed(data, final)
        finally:
            stop_reading.set()
            if rt.is_alive():
                rt.join()
            pi.close()

    def _run_bgzf(self, first: bytes):
        cbuf = np.frombuffer(first, np.uint8)
        in_base = 0                                      # compressed offset of cbuf[0]
        eof = len(first) == 0
        o0 = 0
        last_point = None
        prev_byte = -1
        pending = None                                   # (in_off, in_len, out_len) not yet placed
        while True:
            if not eof and len(cbuf) < BGZF_BATCH:
                more = self.read(BGZF_BATCH)
                eof = len(more) == 0
                if more:
                    cbuf = np.concatenate((cbuf, np.frombuffer(more, np.uint8)))
            if pending is None:
                a, l, o, used = gzlib.bgzf_scan(cbuf)
                if len(a) == 0:
                    # no complete member: drop the zero padding already skipped, then read on (a member is at
                    # most 64 KiB, so more input always completes one unless the stream ends)
                    if used:
                        cbuf = cbuf[used:].copy()
                        in_base += used
                    if eof:
                        if len(cbuf) and (cbuf != 0).any():
                            raise ValueError("gzip stream: truncated BGZF member")
                        return
                    more = self.read(BGZF_BATCH)
                    eof = len(more) == 0
                    if more:
                        cbuf = np.concatenate((cbuf, np.frombuffer(more, np.uint8)))
                    continue
                pending = (a, l, o, used)
            a, l, o, used = pending
            slot = self._take_slot()
            if slot is None:
                return
            out = self.pieces[slot]
            cum = np.cumsum(o)
            k = int(np.searchsorted(cum, len(out), side="right"))
            if k == 0:
                raise ValueError(f"BGZF member of {int(o[0])} B exceeds the piece buffer ({len(out)} B)")
            out_off = np.concatenate(([0], cum[:k - 1])).astype(np.uint64)
            gzlib.inflate_members(cbuf, a[:k], l[:k], out_off, o[:k], out.ctypes.data, self.threads)
            # member-start access points, at most one per span of inflated bytes
            rows = []
            starts = out_off[:k].astype(np.int64) + o0
            i = 0 if last_point is None else int(np.searchsorted(starts, last_point + self.span))
            while i < k:                                 # greedy: the first member start >= span past the last
                ob = int(starts[i])
                pb = int(out[ob - o0 - 1]) if ob > o0 else prev_byte
                rows.append((in_base + int(a[i]), ob, 0, 1, pb, 0))
                last_point = ob
                i = int(np.searchsorted(starts, last_point + self.span))
            n = int(cum[k - 1])
            if n:
                prev_byte = int(out[n - 1])
            pts = np.array(rows, dtype=gzlib.POINTEX_DTYPE) if rows else np.zeros(0, gzlib.POINTEX_DTYPE)
            self.members += k
            self.ready.put(_Piece(slot, o0, n, pts, b""))
            o0 += n
            if k == len(a):
                cbuf = cbuf[used:].copy()
                in_base += used
                pending = None
            else:
                pending = (a[k:], l[k:], o[k:], used)


def index_stream(ctx: ScanContext, read: Callable[[int], bytes], record_lines: int = 4, span: int = 4 << 20,
                 piece_bytes: int = PIECE_BYTES, n_pieces: int = 3, threads: Optional[int] = None,
                 region_bytes: Optional[int] = None) -> GzIndex:
    """Stream a gzip object (``read(n)`` returns its next compressed bytes, b"" at the end) through the
    inflate → HBM → newline-scan pipeline on ``ctx``'s GPU.  See the module doc.  ``region_bytes``: compressed
    bytes per speculative region of the parallel inflater (default 2 MiB; tests use small ones)."""
    k = int(record_lines)
    pins = [ctx.pinned(f"gzpiece{i}", piece_bytes) for i in range(n_pieces)]
    arrays = [p.array[:piece_bytes] for p in pins]
    d_piece = ctx.workspace("gzpiece", piece_bytes + 64)
    cap = piece_bytes // k + 1024                        # read ends per piece: at most one per k bytes (empty lines)
    d_out = ctx.workspace("gzends", 8 * cap + 16)
    res = GzIndex(ends=tempfile.SpooledTemporaryFile(SPOOL_MEM), windows=tempfile.SpooledTemporaryFile(SPOOL_MEM))
    inf = _Inflater(read, arrays, span, threads or pool_threads(), region_bytes)
    inf.start()
    carry = 0                                            # newlines before the current piece
    n_ends = 0                                           # read ends so far
    win_off = 0
    try:
        while True:
            piece = inf.ready.get()
            if piece is None:
                break
            o0, n = piece.o0, piece.n
            host = arrays[piece.slot]
            ends = np.zeros(0, np.uint64)
            nd = 0
            if n:
                ctx.h2d_async(d_piece.ptr, pins[piece.slot].ptr, n)
                rg = np.array([o0, o0 + n], np.uint64)
                while True:
                    ctx.delim_ranges_async(d_piece.ptr, n, o0, rg, 10, k, 1, carry, d_out.ptr, 1, cap)
                    try:
                        cnt, nd, _ = ctx.delim_ranges_result(1)
                        break
                    except DPCapacityError as e:         # cannot happen with the bound above; grow anyway
                        cap = e.needed
                        d_out = ctx.workspace("gzends", 8 * cap + 16)
                ends = ctx.d2h(np.empty(cnt, np.uint64), d_out.ptr)
            # access points of this piece: line number = 1 + newlines before out_byte
            woff = 0
            for p in piece.points:
                ob = int(p["out_byte"])
                j = int(np.searchsorted(ends, np.uint64(ob), side="right"))   # piece's read ends <= ob
                if j:
                    e = int(ends[j - 1])
                    before = (n_ends + j) * k + int(np.count_nonzero(host[e - o0:ob - o0] == 10))
                else:
                    before = carry + int(np.count_nonzero(host[:ob - o0] == 10))
                wl = int(p["window_len"])
                at_start = ob == 0 or int(p["prev_byte"]) == 10
                res.rows.append([len(res.rows), int(p["in_byte"]), ob, before + 1, wl, win_off, int(p["bits"]),
                                 int(p["member_start"]), int(at_start)])
                if wl:
                    res.windows.write(piece.windows[woff:woff + wl])
                woff += wl
                win_off += wl
            if len(ends):
                res.ends.write(np.ascontiguousarray(ends, "<u8").tobytes())
            if n:
                res.last_byte = int(host[n - 1])
            n_ends += len(ends)
            carry += nd
            res.uncompressed_size = o0 + n
            res.pieces += 1
            inf.free.put(piece.slot)                     # the piece's bytes are no longer needed
    finally:
        inf.stop.set()
        inf.join()
    if inf.error is not None:
        raise inf.error
    res.newlines = carry
    res.num_records = n_ends
    res.members = inf.members
    res.bgzf = inf.bgzf
    res.ends.seek(0)
    res.windows.seek(0)
    return res
