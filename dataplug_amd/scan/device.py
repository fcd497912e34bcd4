"""Device-side scan contexts: one ``dp_ctx`` (device + HIP stream + workspace) per host thread per GPU.

This is the only Python module that talks to libdpscan.so.  Buffers handed to the kernels are device
pointers (ints): either the context's own grow-only staging buffers (``*_host`` helpers upload Python
bytes / numpy arrays), or caller-owned device memory (e.g. a torch tensor's ``data_ptr()``).
"""
from __future__ import annotations

import ctypes
import threading
from typing import Iterable, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import DPCapacityError, check

_U64P = ctypes.POINTER(ctypes.c_uint64)
_I64P = ctypes.POINTER(ctypes.c_int64)


def _host_ptr(data) -> Tuple[int, int, object]:
    """(address, nbytes, keepalive) of a bytes-like / numpy object without copying."""
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    else:
        a = np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)
    return a.ctypes.data, a.nbytes, a


class DeviceBuffer:
    """Device memory owned through the C ABI (freed with the context)."""

    def __init__(self, ctx: "ScanContext", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(_lib.load().dp_malloc(ctx.handle, max(16, self.nbytes), ctypes.byref(p)))
        self.ptr = int(p.value)

    def free(self):
        if self.ptr and self.ctx.handle:
            check(_lib.load().dp_free(self.ctx.handle, ctypes.c_void_p(self.ptr)))
        self.ptr = 0


class PinnedBuffer:
    """Page-locked host memory (dp_host_alloc) with a uint8 numpy view; H2D from it is a true async DMA."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(_lib.load().dp_host_alloc(max(16, self.nbytes), ctypes.byref(p)))
        self.ptr = int(p.value)
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(16, self.nbytes)).from_address(self.ptr))

    def view(self, n: Optional[int] = None) -> memoryview:
        return memoryview(self.array)[: self.nbytes if n is None else n]

    def free(self):
        if self.ptr:
            self.array = None
            check(_lib.load().dp_host_free(ctypes.c_void_p(self.ptr)))
        self.ptr = 0


# Placement-aware input buffers (round 6, profiles/r06/placement/): about half of the large device buffers a process
# allocates sit in a "slow mode" where a kernel reading the buffer while writing a few % of its size elsewhere runs
# 10-16 % slower than on the other half (reads alone are not affected; the input buffer alone decides, whatever the
# output buffer).  An input buffer of at least PLACEMENT_MIN bytes is therefore probed when it is allocated: the
# calibration kernels read it alone and read it while writing 1/32 of it; a time ratio above PLACEMENT_SLOW marks the
# slow mode, and another buffer is allocated (the slow one held meanwhile, so it is not handed back) -- at most
# PLACEMENT_TRIES, the best kept (or the best of those that fit in HBM).  Eight 4 GiB buffers of one process
# (tools/placement_probe.py, profiles/r06/placement/probe8.log): ratios 1.088-1.106 where line_kernel's u8s scan of a
# 4 GiB CSV takes 688-700 us, 1.167-1.193 where it takes 787-792 us (8 GiB: 1.080-1.094 / 1,352-1,356 us against
# 1.184-1.199 / 1,567-1,569 us, probe8g.log).  Larger buffers are mixtures (four 32 GiB
# ones: ratios 1.055-1.108 against scans of 6,006-6,302 us, no separation; profiles/r06/placement/probe32.log), so
# buffers above PLACEMENT_MAX are allocated once, unprobed.
PLACEMENT_MIN = 256 << 20
PLACEMENT_MAX = 8 << 30
PLACEMENT_TRIES = 5
PLACEMENT_SLOW = 1.125
_PROBE_WPR = 1.0 / 32


class ScanContext:
    """A ``dp_ctx``: device, stream and scan workspace.  Not shared between threads."""

    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        h = ctypes.c_void_p()
        check(self.lib.dp_ctx_create(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = int(device)
        self._bufs = {}
        self._pinned = {}
        self._get_pool = None
        self._timing_on = False
        self.placements = []                          # per placed buffer: the probe ratios of its candidates

    # ---------------------------------------------------------------- memory
    def workspace(self, name: str, nbytes: int, placed: bool = False) -> DeviceBuffer:
        """Grow-only named device buffer; ``placed``: an input buffer, probed for the slow placement mode when it is
        allocated (``PLACEMENT_MIN`` .. ``PLACEMENT_MAX`` bytes)."""
        b = self._bufs.get(name)
        if b is None or b.nbytes < nbytes:
            if b is not None:
                b.free()
                del self._bufs[name]
            size = max(int(nbytes), 1 << 16)
            b = (self._placed_buffer(size) if placed and PLACEMENT_MIN <= size <= PLACEMENT_MAX
                 else DeviceBuffer(self, size))
            self._bufs[name] = b
        return b

    def placement_ratio(self, buf: DeviceBuffer, nbytes: Optional[int] = None) -> float:
        """Time of the read-while-writing calibration kernel over ``buf`` / time of the read-only one (each the
        mean of two launches): ~1.0-1.03 on a fast buffer, ~1.08-1.16 in the slow mode."""
        n = (buf.nbytes if nbytes is None else nbytes) // 16 * 16
        out = DeviceBuffer(self, int(n * _PROBE_WPR) + (1 << 16))
        was_on = self._timing_on
        try:
            self.stream_read(buf.ptr, n)
            self.sync()
            t = []
            for rw in (False, True):
                self.timing(True)
                self.timing_read()
                for _ in range(2):
                    if rw:
                        self.stream_rw(buf.ptr, n, out.ptr, _PROBE_WPR)
                    else:
                        self.stream_read(buf.ptr, n)
                ms, k = self.timing_read()
                t.append(ms / max(1, k))
            return t[1] / t[0]
        finally:
            self.timing(was_on)
            out.free()

    def _placed_buffer(self, size: int) -> DeviceBuffer:
        cands = []
        try:
            for _ in range(PLACEMENT_TRIES):
                try:
                    c = DeviceBuffer(self, size)
                except _lib.DPScanError:
                    if cands:                         # no room for another candidate: the best so far
                        break
                    raise
                cands.append((self.placement_ratio(c), c))
                if cands[-1][0] <= PLACEMENT_SLOW:
                    break
        except BaseException:
            for _, c in cands:
                c.free()
            raise
        best = min(cands, key=lambda rc: rc[0])
        for rc in cands:
            if rc is not best:
                rc[1].free()
        self.placements.append([round(r, 4) for r, _ in cands])
        return best[1]

    def pinned(self, name: str, nbytes: int) -> PinnedBuffer:
        """Grow-only named pinned host buffer."""
        b = self._pinned.get(name)
        if b is None or b.nbytes < nbytes:
            if b is not None:
                b.free()
            b = PinnedBuffer(max(int(nbytes), 1 << 16))
            self._pinned[name] = b
        return b

    def get_pool(self, threads: int):
        """The context's persistent pool of ranged-GET threads (``fetch_to_device``): created once per context,
        i.e. once per (host thread, device) — a persistent per-GPU worker reuses it for every object."""
        import concurrent.futures as cf
        if self._get_pool is None or self._get_pool._max_workers < threads:
            if self._get_pool is not None:
                self._get_pool.shutdown(wait=True)
            self._get_pool = cf.ThreadPoolExecutor(threads, thread_name_prefix=f"dpscan-get{self.device}")
        return self._get_pool

    def h2d_async(self, dst: int, src_ptr: int, nbytes: int) -> None:
        """Async copy from pinned host memory on the context stream (caller keeps the source alive)."""
        check(self.lib.dp_h2d(self.handle, ctypes.c_void_p(dst), ctypes.c_void_p(src_ptr), int(nbytes)))

    def h2d(self, dst: int, data, nbytes: Optional[int] = None) -> None:
        ptr, n, keep = _host_ptr(data)
        n = n if nbytes is None else nbytes
        check(self.lib.dp_h2d(self.handle, ctypes.c_void_p(dst), ctypes.c_void_p(ptr), n))
        check(self.lib.dp_sync(self.handle))   # pageable source: keep it alive until the copy is done
        del keep

    def d2h_async(self, dst_ptr: int, src: int, nbytes: int) -> None:
        """Async copy to pinned host memory on the context stream (ordered after the work enqueued before it)."""
        if nbytes:
            check(self.lib.dp_d2h(self.handle, ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src), int(nbytes)))

    def d2h(self, out: np.ndarray, src: int) -> np.ndarray:
        if out.nbytes:
            check(self.lib.dp_d2h(self.handle, ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(src), out.nbytes))
            check(self.lib.dp_sync(self.handle))
        return out

    def upload(self, data, name: str = "input") -> Tuple[int, int]:
        """Copy host bytes into the named staging buffer; returns (device pointer, nbytes)."""
        _, n, _ = _host_ptr(data)
        buf = self.workspace(name, n + 16)
        self.h2d(buf.ptr, data)
        return buf.ptr, n

    def sync(self) -> None:
        check(self.lib.dp_sync(self.handle))

    @property
    def stream(self) -> int:
        s = ctypes.c_void_p()
        check(self.lib.dp_ctx_get_stream(self.handle, ctypes.byref(s)))
        return int(s.value or 0)

    def set_stream(self, stream: Optional[int]) -> None:
        check(self.lib.dp_ctx_set_stream(self.handle, ctypes.c_void_p(stream or 0)))

    def wait_for(self, other: "ScanContext") -> None:
        """This context's stream waits (on the device) for everything enqueued on ``other``'s so far."""
        check(self.lib.dp_ctx_wait(self.handle, other.handle))

    # ---------------------------------------------------------------- FASTA
    def fasta_index(self, d_buf: int, buf_len: int, buf_base: int, obj_size: int,
                    chunks: Sequence[Tuple[int, int]], u64: bool = False, cap: Optional[int] = None):
        """FASTA (start, end) pairs of a chunk plan over device bytes (dp_fasta_index).

        Returns (pairs (n, 2) uint32|uint64, pending (nchunks,) int64, chunk_end (nchunks,) uint64).
        """
        ch = np.ascontiguousarray(np.asarray(chunks, dtype=np.uint64).reshape(-1))
        nch = len(ch) // 2
        dtype = np.uint64 if u64 else np.uint32
        if cap is None:
            cap = buf_len // 512 + 1024
        pending = np.full(nch, -1, np.int64)
        cend = np.zeros(nch, np.uint64)
        n = ctypes.c_uint64(0)
        while True:
            out = self.workspace("out", 2 * cap * np.dtype(dtype).itemsize + 16)
            rc = self.lib.dp_fasta_index(self.handle, ctypes.c_void_p(d_buf), buf_len, buf_base, obj_size,
                                         ch.ctypes.data_as(_U64P), nch, ctypes.c_void_p(out.ptr), int(u64), cap,
                                         ctypes.byref(n), pending.ctypes.data_as(_I64P), cend.ctypes.data_as(_U64P))
            if rc == _lib.DP_ERR_CAPACITY:
                cap = int(n.value)
                continue
            check(rc)
            break
        pairs = self.d2h(np.empty((int(n.value), 2), dtype), out.ptr)
        return pairs, pending, cend

    def fasta_index_async(self, d_buf, buf_len, buf_base, obj_size, chunks_u64: np.ndarray, d_out: int,
                          u64: bool, cap: int) -> None:
        check(self.lib.dp_fasta_index_async(self.handle, ctypes.c_void_p(d_buf), buf_len, buf_base, obj_size,
                                            chunks_u64.ctypes.data_as(_U64P), len(chunks_u64) // 2,
                                            ctypes.c_void_p(d_out), int(u64), cap))

    def fasta_result(self, nchunks: int):
        n = ctypes.c_uint64(0)
        pending = np.full(nchunks, -1, np.int64)
        cend = np.zeros(nchunks, np.uint64)
        check(self.lib.dp_fasta_result(self.handle, ctypes.byref(n), pending.ctypes.data_as(_I64P),
                                       cend.ctypes.data_as(_U64P)))
        return int(n.value), pending, cend

    # ---------------------------------------------------------------- delimiters
    def delim_index(self, d_buf: int, buf_len: int, buf_base: int, begin: int, end: int, delim: int = 10,
                    every_k: int = 1, emit_add: int = 0, u64: bool = True, cap: Optional[int] = None):
        """Sorted offsets of every ``every_k``-th ``delim`` in object bytes [begin, end) (dp_delim_index).

        Returns (offsets uint64|uint32, number of delimiters seen)."""
        dtype = np.uint64 if u64 else np.uint32
        if cap is None:
            cap = (end - begin) // (16 * every_k) + 1024
        n = ctypes.c_uint64(0)
        nd = ctypes.c_uint64(0)
        while True:
            out = self.workspace("out", cap * np.dtype(dtype).itemsize + 16)
            rc = self.lib.dp_delim_index(self.handle, ctypes.c_void_p(d_buf), buf_len, buf_base, begin, end,
                                         int(delim), int(every_k), int(emit_add), ctypes.c_void_p(out.ptr),
                                         int(u64), cap, ctypes.byref(n), ctypes.byref(nd))
            if rc == _lib.DP_ERR_CAPACITY:
                cap = int(n.value)
                continue
            check(rc)
            break
        return self.d2h(np.empty(int(n.value), dtype), out.ptr), int(nd.value)

    def delim_index_async(self, d_buf, buf_len, buf_base, begin, end, delim, every_k, emit_add, d_out, u64, cap):
        check(self.lib.dp_delim_index_async(self.handle, ctypes.c_void_p(d_buf), buf_len, buf_base, begin, end,
                                            int(delim), int(every_k), int(emit_add), ctypes.c_void_p(d_out),
                                            int(u64), cap))

    def delim_result(self):
        n = ctypes.c_uint64(0)
        nd = ctypes.c_uint64(0)
        check(self.lib.dp_delim_result(self.handle, ctypes.byref(n), ctypes.byref(nd)))
        return int(n.value), int(nd.value)

    def delim_ranges_async(self, d_buf: int, buf_len: int, buf_base: int, ranges: np.ndarray, delim: int,
                           every_k: int, emit_add: int, carry: int, d_out: int, out_mode: int, cap: int) -> None:
        """dp_delim_ranges_async; ``ranges`` a contiguous uint64 array [lo0, hi0, lo1, hi1, ...] kept alive by
        the caller until the result is collected."""
        check(self.lib.dp_delim_ranges_async(self.handle, ctypes.c_void_p(d_buf), buf_len, buf_base,
                                             ranges.ctypes.data_as(_U64P), len(ranges) // 2, int(delim),
                                             int(every_k), int(emit_add), int(carry), ctypes.c_void_p(d_out),
                                             int(out_mode), int(cap)))

    def delim_ranges_result(self, nranges: int):
        """(entries, delimiters seen, per-range cumulative delimiter counts)."""
        n = ctypes.c_uint64(0)
        nd = ctypes.c_uint64(0)
        ends = np.zeros(nranges, np.uint64)
        rc = self.lib.dp_delim_ranges_result(self.handle, ctypes.byref(n), ctypes.byref(nd), ends.ctypes.data_as(_U64P))
        if rc == _lib.DP_ERR_CAPACITY:
            e = DPCapacityError(rc, f"output capacity below {int(n.value)} entries")
            e.needed = int(n.value)
            raise e
        check(rc)
        return int(n.value), int(nd.value), ends

    @staticmethod
    def block_table_size(ranges: np.ndarray) -> Tuple[int, int]:
        """(j0, entries) of the 64 KiB block table out_mode 3 writes for these ranges."""
        first, last = int(ranges[0]), int(ranges[-1])
        j0 = first >> 16
        return j0, (((last - 1) >> 16) - j0 + 1) if last > first else 1

    @staticmethod
    def sub_table_size(ranges: np.ndarray) -> Tuple[int, int]:
        """(s0, entries) of the 256-byte table out_mode 4 writes for these ranges."""
        first, last = int(ranges[0]), int(ranges[-1])
        s0 = first >> 8
        return s0, (((last - 1) >> 8) - s0 + 1) if last > first else 1

    @staticmethod
    def _tab_off(cap: int, out_mode: int) -> int:
        return ((2 if out_mode == 3 else 1) * cap + 15) & ~15

    @staticmethod
    def _sub_off(cap: int, ranges: np.ndarray) -> int:
        return (ScanContext._tab_off(cap, 4) + 8 * ScanContext.block_table_size(ranges)[1] + 15) & ~15

    @staticmethod
    def out_bytes(cap: int, out_mode: int, ranges: np.ndarray) -> int:
        """Bytes of a dp_delim_ranges output buffer for ``cap`` entries (out_mode 3: + the block table; 4: + the
        block table and the 256-byte table)."""
        if out_mode == 3:
            return ScanContext._tab_off(cap, 3) + 8 * ScanContext.block_table_size(ranges)[1] + 16
        if out_mode == 4:
            return ScanContext._sub_off(cap, ranges) + 2 * ScanContext.sub_table_size(ranges)[1] + 16
        return cap * (8 if out_mode == 1 else 4) + 16

    def block_table(self, d_out: int, cap: int, ranges: np.ndarray, out_mode: int = 3) -> np.ndarray:
        """The 64 KiB block table of an out_mode 3 / 4 result: entries before (j0 + j) * 64 KiB (this launch)."""
        j0, nt = self.block_table_size(ranges)
        tab = self.d2h(np.empty(nt, np.uint64), d_out + self._tab_off(cap, out_mode))
        if int(ranges[0]) & 0xFFFF:
            tab[0] = 0                                   # the boundary below the first byte: not a range start
        return tab

    def sub_table(self, d_out: int, cap: int, ranges: np.ndarray) -> np.ndarray:
        """The 256-byte table of an out_mode 4 result: low 16 bits of the entries before (s0 + s) * 256."""
        s0, ns = self.sub_table_size(ranges)
        sub = self.d2h(np.empty(ns, np.uint16), d_out + self._sub_off(cap, ranges))
        if int(ranges[0]) & 0xFF:
            sub[0] = 0                                   # the boundary below the first byte
        return sub

    def delim_ranges(self, d_buf: int, buf_len: int, buf_base: int, ranges, delim: int = 10, every_k: int = 1,
                     emit_add: int = 0, carry: int = 0, out_mode: int = 1, cap: Optional[int] = None):
        """Synchronous dp_delim_ranges: (offsets, delimiters seen, per-range cumulative counts); out_mode 1
        uint64, 0 uint32, 2 uint32 low words, 3 uint16 low words (+ ``block_table``, returned as a 4th item), 4 uint8
        low bytes (+ ``block_table`` and ``sub_table``, a 4th and 5th item)."""
        rg = np.ascontiguousarray(np.asarray(ranges, dtype=np.uint64).reshape(-1))
        span = int(sum(int(rg[2 * i + 1]) - int(rg[2 * i]) for i in range(len(rg) // 2)))
        dtype = {0: np.uint32, 1: np.uint64, 2: np.uint32, 3: np.uint16, 4: np.uint8}[out_mode]
        if cap is None:
            cap = span // (16 * every_k) + 1024
        while True:
            out = self.workspace("out", self.out_bytes(cap, out_mode, rg))
            self.delim_ranges_async(d_buf, buf_len, buf_base, rg, delim, every_k, emit_add, carry, out.ptr,
                                    out_mode, cap)
            try:
                n, nd, ends = self.delim_ranges_result(len(rg) // 2)
            except DPCapacityError as e:
                cap = e.needed
                continue
            vals = self.d2h(np.empty(n, dtype), out.ptr)
            if out_mode == 3:
                return vals, nd, ends, self.block_table(out.ptr, cap, rg)
            if out_mode == 4:
                return vals, nd, ends, self.block_table(out.ptr, cap, rg, 4), self.sub_table(out.ptr, cap, rg)
            return vals, nd, ends

    def find_delim(self, d_buf: int, buf_len: int, buf_base: int, start: int, delim: int = 10) -> int:
        """First object offset >= start holding ``delim`` in the buffer, or -1."""
        pos = ctypes.c_int64(-1)
        check(self.lib.dp_find_delim(self.handle, ctypes.c_void_p(d_buf), buf_len, buf_base, start, int(delim),
                                     ctypes.byref(pos)))
        return int(pos.value)

    # ---------------------------------------------------------------- host-buffer conveniences
    def fasta_index_host(self, data, buf_base: int, obj_size: int, chunks, u64: bool = False):
        ptr, n = self.upload(data)
        return self.fasta_index(ptr, n, buf_base, obj_size, chunks, u64=u64)

    def delim_index_host(self, data, buf_base: int, begin: int, end: int, **kw):
        ptr, n = self.upload(data)
        return self.delim_index(ptr, n, buf_base, begin, end, **kw)

    def find_delim_host(self, data, buf_base: int, start: int, delim: int = 10) -> int:
        ptr, n = self.upload(data, name="halo")
        return self.find_delim(ptr, n, buf_base, start, delim)

    def stream_read(self, d_buf: int, nbytes: int, blocks_per_cu: int = 0) -> None:
        """Calibration read of ``nbytes`` device bytes (async; time it with timing())."""
        check(self.lib.dp_stream_read(self.handle, ctypes.c_void_p(d_buf), nbytes, blocks_per_cu))

    def stream_rw(self, d_in: int, nbytes: int, d_out: int, write_per_read: float, blocks_per_cu: int = 0) -> None:
        """Calibration read of ``nbytes`` plus ``write_per_read * nbytes`` contiguous output bytes (async)."""
        q = int(round(write_per_read * 65536))
        check(self.lib.dp_stream_rw(self.handle, ctypes.c_void_p(d_in), nbytes, ctypes.c_void_p(d_out if q else 0),
                                    q, blocks_per_cu))

    # ---------------------------------------------------------------- timing / geometry
    def timing(self, enable: bool) -> None:
        check(self.lib.dp_timing_enable(self.handle, int(bool(enable))))
        self._timing_on = bool(enable)

    def timing_read(self) -> Tuple[float, int]:
        ms = ctypes.c_double(0.0)
        n = ctypes.c_uint64(0)
        check(self.lib.dp_timing_read(self.handle, ctypes.byref(ms), ctypes.byref(n)))
        return float(ms.value), int(n.value)

    _FORM_KEYS = {"fasta": _lib.DP_FORM_FASTA, "delim": _lib.DP_FORM_DELIM,
                  "delim_line_max": _lib.DP_FORM_DELIM_LINE_MAX, "delim_dense": _lib.DP_FORM_DELIM_DENSE}

    def set_form(self, **kw) -> None:
        """dp_ctx_set_form: fasta=0 (map + placement, default) | 1 (one-pass); delim=0 (auto, default) | 1 (line) |
        3 (one-pass); delim_line_max=bytes; delim_dense=delimiters per KiB x 1000.  The shipped
        defaults need no call; tests and A/B runs pin a form with it."""
        for k, v in kw.items():
            check(self.lib.dp_ctx_set_form(self.handle, self._FORM_KEYS[k], int(v)))

    def get_form(self, key: str) -> int:
        v = ctypes.c_uint64(0)
        check(self.lib.dp_ctx_get_form(self.handle, self._FORM_KEYS[key], ctypes.byref(v)))
        return int(v.value)

    DELIM_FORMS = {0: "auto: the density probe picks per launch",
                   1: "line_kernel<DELIM> (lockstep one pass)",
                   3: "scan_kernel<DELIM> (one-pass look-back)"}

    def delim_form(self, span: int, out_mode: int = 3) -> int:
        """The kernels a newline launch of ``span`` bytes into ``out_mode`` takes (dp_scan_delim_form: 1 line,
        3 one-pass; 0: the launch's own bytes decide on the device)."""
        f = ctypes.c_int(0)
        check(self.lib.dp_scan_delim_form(self.handle, int(span), int(out_mode), ctypes.byref(f)))
        return int(f.value)

    def last_delim_form(self) -> int:
        """The kernels the last collected newline launch ran (dp_last_delim_form: 1 or 3; 0 before any)."""
        f = ctypes.c_int(0)
        check(self.lib.dp_last_delim_form(self.handle, ctypes.byref(f)))
        return int(f.value)

    def geometry(self) -> Tuple[int, int]:
        g = ctypes.c_int(0)
        u = ctypes.c_int(0)
        check(self.lib.dp_scan_geometry(self.handle, ctypes.byref(g), ctypes.byref(u)))
        return int(g.value), int(u.value)

    def close(self) -> None:
        if self._get_pool is not None:
            self._get_pool.shutdown(wait=True)
            self._get_pool = None
        if self.handle:
            for b in list(self._bufs.values()) + list(self._pinned.values()):
                b.free()
            self._bufs.clear()
            self._pinned.clear()
            check(self.lib.dp_ctx_destroy(self.handle))
            self.handle = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass


_tls = threading.local()


def device_count() -> int:
    return _lib.device_count()


def get_context(device: int = 0, slot: int = 0) -> ScanContext:
    """The calling thread's context for ``device`` (created on first use); ``slot`` > 0 names further contexts of
    the thread on the same device (their own stream and buffers: a thread alternating two overlaps one's copies with
    the other's scan)."""
    ctxs = getattr(_tls, "ctxs", None)
    if ctxs is None:
        ctxs = _tls.ctxs = {}
    key = device if slot == 0 else (device, slot)
    c = ctxs.get(key)
    if c is None:
        c = ctxs[key] = ScanContext(device)
    return c


def close_context(device: int = 0) -> None:
    """Close the calling thread's contexts for ``device``, if any (their streams, pinned staging and HBM workspaces
    are freed; the next ``get_context`` makes new ones)."""
    ctxs = getattr(_tls, "ctxs", {})
    for key in [k for k in ctxs if k == device or (isinstance(k, tuple) and k[0] == device)]:
        ctxs.pop(key).close()


def pick_device(i: int, devices: Optional[Iterable[int]] = None) -> int:
    """Round-robin device for job ``i`` over ``devices`` (default: every visible GPU)."""
    devs = list(devices) if devices is not None else list(range(max(1, device_count())))
    return devs[i % len(devs)]
