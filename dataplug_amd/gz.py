"""Gzip access points: build (libdpgz.so, zlib Z_BLOCK) and resume inflating mid-stream.

What gztool's index gives the reference (dataplug/formats/compressed/gzipped.py:46-153, 268-354): start
inflating at a point inside the compressed object instead of at byte 0.  A point is
(in_byte, bits, out_byte, member_start); resuming needs the 32 KiB of output before out_byte (the window).
Deflate blocks start at arbitrary bit offsets: the compressed bytes from in_byte-1 are shifted by ``bits``
so the block starts at bit 0, then inflated raw with the window as the zlib dictionary.
"""
from __future__ import annotations

import ctypes
import os
import zlib
from typing import Callable, Iterable, Iterator, Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPGZ_LIB", os.path.join(_HERE, "lib", "libdpgz.so"))
WINDOW = 32768

POINT_DTYPE = np.dtype([("in_byte", "<u8"), ("out_byte", "<u8"), ("bits", "<u4"), ("member_start", "<u4")])


class _Point(ctypes.Structure):
    _fields_ = [("in_byte", ctypes.c_uint64), ("out_byte", ctypes.c_uint64), ("bits", ctypes.c_uint32),
                ("member_start", ctypes.c_uint32)]


class _Result(ctypes.Structure):
    _fields_ = [("out", ctypes.POINTER(ctypes.c_uint8)), ("out_len", ctypes.c_uint64),
                ("points", ctypes.POINTER(_Point)), ("n_points", ctypes.c_uint64), ("members", ctypes.c_uint64)]


POINTEX_DTYPE = np.dtype([("in_byte", "<u8"), ("out_byte", "<u8"), ("bits", "<u4"), ("member_start", "<u4"),
                          ("prev_byte", "<i4"), ("window_len", "<u4")])

_lib = None
_ERRORS = {1: "invalid argument", 2: "out of memory", 3: "corrupt gzip/deflate data", 4: "truncated gzip stream"}
_U64P = ctypes.POINTER(ctypes.c_uint64)


def _check(rc: int, what: str) -> None:
    if rc:
        raise ValueError(f"{what}: {_ERRORS.get(rc, rc)}")


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not found: build it with `python -m dataplug_amd.build`")
        lib = ctypes.CDLL(LIB_PATH)
        lib.dpgz_build.restype = ctypes.c_int
        lib.dpgz_build.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                   ctypes.POINTER(ctypes.POINTER(_Result))]
        lib.dpgz_free.restype = None
        lib.dpgz_free.argtypes = [ctypes.POINTER(_Result)]
        lib.dpgz_abi_version.restype = ctypes.c_int
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        lib.dpgz_stream_new.restype = ctypes.c_int
        lib.dpgz_stream_new.argtypes = [u64, ctypes.POINTER(vp)]
        lib.dpgz_stream_free.restype = None
        lib.dpgz_stream_free.argtypes = [vp]
        lib.dpgz_stream_inflate.restype = ctypes.c_int
        lib.dpgz_stream_inflate.argtypes = [vp, vp, u64, ctypes.c_int, vp, u64, _U64P, _U64P,
                                            ctypes.POINTER(ctypes.c_int)]
        lib.dpgz_stream_take.restype = ctypes.c_int
        lib.dpgz_stream_take.argtypes = [vp, vp, u64, vp, u64, _U64P, _U64P]
        lib.dpgz_stream_state.restype = ctypes.c_int
        lib.dpgz_stream_state.argtypes = [vp, _U64P, _U64P, _U64P, _U64P, _U64P]
        lib.dpgz_bgzf_scan.restype = ctypes.c_int
        lib.dpgz_bgzf_scan.argtypes = [vp, u64, _U64P, _U64P, _U64P, u64, _U64P, _U64P]
        lib.dpgz_inflate_members.restype = ctypes.c_int
        lib.dpgz_inflate_members.argtypes = [vp, _U64P, _U64P, _U64P, _U64P, u64, vp, ctypes.c_int]
        lib.dpgz_par_new.restype = ctypes.c_int
        lib.dpgz_par_new.argtypes = [u64, ctypes.c_int, ctypes.POINTER(vp)]
        lib.dpgz_par_free.restype = None
        lib.dpgz_par_free.argtypes = [vp]
        lib.dpgz_par_set_region.restype = ctypes.c_int
        lib.dpgz_par_set_region.argtypes = [vp, u64]
        lib.dpgz_par_feed.restype = ctypes.c_int
        lib.dpgz_par_feed.argtypes = [vp, vp, u64, ctypes.c_int]
        lib.dpgz_par_read.restype = ctypes.c_int
        lib.dpgz_par_read.argtypes = [vp, vp, u64, _U64P]
        lib.dpgz_par_take.restype = ctypes.c_int
        lib.dpgz_par_take.argtypes = [vp, u64, vp, u64, vp, u64, _U64P, _U64P]
        lib.dpgz_par_state.restype = ctypes.c_int
        lib.dpgz_par_state.argtypes = [vp, _U64P]
        if lib.dpgz_abi_version() < 3:
            raise ImportError(f"{LIB_PATH} is out of date: rebuild it with `python -m dataplug_amd.build`")
        _lib = lib
    return _lib


def build_index(gz, span: int = 1 << 20, out_hint: int = 0):
    """(inflated bytes as a uint8 array, access points as a POINT_DTYPE array)."""
    src = np.frombuffer(memoryview(gz).cast("B"), np.uint8)
    res = ctypes.POINTER(_Result)()
    rc = load().dpgz_build(src.ctypes.data, len(src), int(span), int(out_hint), ctypes.byref(res))
    if rc:
        raise ValueError(f"gzip index: {_ERRORS.get(rc, rc)}")
    try:
        r = res.contents
        out = np.ctypeslib.as_array(r.out, shape=(r.out_len,)).copy() if r.out_len else np.zeros(0, np.uint8)
        pts = np.zeros(r.n_points, POINT_DTYPE)
        if r.n_points:
            raw = np.ctypeslib.as_array(ctypes.cast(r.points, ctypes.POINTER(ctypes.c_uint8)),
                                        shape=(r.n_points * POINT_DTYPE.itemsize,))
            pts = raw.view(POINT_DTYPE).copy()
    finally:
        load().dpgz_free(res)
    return out, pts


class _Shifter:
    """Streams bytes x0 x1 x2 ... as y_i = (x_i >> (8 - b)) | (x_{i+1} << b): the bit stream starting at
    the top ``b`` bits of x0."""

    def __init__(self, b: int):
        self.b = b
        self.prev: Optional[int] = None

    def feed(self, chunk: bytes) -> bytes:
        if self.b == 0:
            return chunk
        x = np.frombuffer(chunk, np.uint8).astype(np.uint16)
        if self.prev is not None:
            x = np.concatenate(([self.prev], x))
        if len(x) < 2:
            self.prev = int(x[0]) if len(x) else self.prev
            return b""
        y = ((x[:-1] >> (8 - self.b)) | (x[1:] << self.b)) & 0xFF
        self.prev = int(x[-1])
        return y.astype(np.uint8).tobytes()

    def flush(self) -> bytes:
        if self.b == 0 or self.prev is None:
            return b""
        return bytes([self.prev >> (8 - self.b)])


def _members_from(src: Iterable[bytes]) -> Iterator[bytes]:
    """Inflate consecutive gzip members from a compressed byte stream that starts at a member start
    (zero padding between members tolerated), to the end of the stream."""
    d = None
    for c in src:
        while c:
            if d is None:
                c = c.lstrip(b"\0")
                if not c:
                    break
                d = zlib.decompressobj(wbits=31)
            out = d.decompress(c)
            if out:
                yield out
            if d.eof:
                c = d.unused_data
                d = None
            else:
                c = b""
    if d is not None:
        tail = d.flush()
        if tail:
            yield tail
        if not d.eof:
            raise ValueError("gzip stream: truncated member")


def inflate_from(points: np.ndarray, i: int, window: bytes, fetch: Callable[[int], Iterable[bytes]]) -> Iterator[bytes]:
    """Inflated bytes from access point ``i`` to the end of the object.

    ``fetch(offset)`` yields the compressed object's bytes from ``offset`` onwards (chunks of any size;
    the caller may stop iterating any time).  From a member-start point the members that follow are inflated
    in sequence from the same bytes (BGZF indexes keep only some member starts as points).  From a point
    inside a member, the member's end is not byte-addressable in the shifted stream, so the stream continues
    at the next member-start point (streams indexed block-wise keep every member start as a point)."""
    while i < len(points):
        p = points[i]
        if p["member_start"]:
            yield from _members_from(fetch(int(p["in_byte"])))
            return
        b = int(p["bits"])
        d = zlib.decompressobj(wbits=-15, zdict=window) if window else zlib.decompressobj(wbits=-15)
        src = fetch(int(p["in_byte"]) - (1 if b else 0))
        sh = _Shifter(b)
        for c in src:
            c = sh.feed(c)
            out = d.decompress(c)
            if out:
                yield out
            if d.eof:
                break
        else:
            if not d.eof:
                out = d.decompress(sh.flush())
                if out:
                    yield out
            tail = d.flush()
            if tail:
                yield tail
        if not d.eof:
            return
        # next member: the first member-start point after this one
        j = i + 1
        while j < len(points) and not points[j]["member_start"]:
            j += 1
        i = j
        window = b""


def window_of(inflated: np.ndarray, out_byte: int) -> bytes:
    return inflated[max(0, out_byte - WINDOW):out_byte].tobytes()


# ------------------------------------------------------------------------------------------ streaming
def _addr(buf) -> int:
    """Address of a writable/readable contiguous buffer (numpy array, bytearray, bytes, memoryview)."""
    if isinstance(buf, np.ndarray):
        return buf.ctypes.data
    return np.frombuffer(buf, np.uint8).ctypes.data if len(buf) else 0


class InflateStream:
    """libdpgz's streaming inflater: compressed bytes in as they arrive, inflated bytes out into the caller's
    buffer, access points (with their windows) collected on the way (see include/dpgz.h)."""

    def __init__(self, span: int = 1 << 20):
        h = ctypes.c_void_p()
        _check(load().dpgz_stream_new(int(span), ctypes.byref(h)), "gzip stream")
        self._h = h

    def inflate(self, data, final: bool, out: np.ndarray, out_off: int, out_cap: int):
        """(consumed, produced, at_end): inflate ``data`` into out[out_off : out_off + out_cap]."""
        c, p, e = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_int(0)
        keep = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
        _check(load().dpgz_stream_inflate(self._h, keep.ctypes.data, len(data), int(final),
                                          out.ctypes.data + out_off, int(out_cap), ctypes.byref(c), ctypes.byref(p),
                                          ctypes.byref(e)), "gzip stream")
        return int(c.value), int(p.value), bool(e.value)

    def take(self):
        """(points as a POINTEX_DTYPE array, their windows concatenated as bytes) found since the last take."""
        st = [ctypes.c_uint64(0) for _ in range(5)]
        load().dpgz_stream_state(self._h, *[ctypes.byref(x) for x in st])
        npts, nwin = int(st[3].value), int(st[4].value)
        pts = np.zeros(npts, POINTEX_DTYPE)
        win = np.zeros(max(1, nwin), np.uint8)
        n, w = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _check(load().dpgz_stream_take(self._h, pts.ctypes.data if npts else None, npts, win.ctypes.data, nwin,
                                       ctypes.byref(n), ctypes.byref(w)), "gzip stream")
        return pts[: int(n.value)], win[: int(w.value)].tobytes()

    def state(self):
        """(compressed bytes consumed, inflated bytes produced, members started)."""
        st = [ctypes.c_uint64(0) for _ in range(5)]
        load().dpgz_stream_state(self._h, *[ctypes.byref(x) for x in st])
        return int(st[0].value), int(st[1].value), int(st[2].value)

    def close(self):
        if self._h:
            load().dpgz_stream_free(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class ParInflate:
    """libdpgz's parallel inflater of one gzip stream (include/dpgz.h, csrc/dpgz_par.c): compressed bytes in,
    inflated bytes out in order, the same access points as InflateStream, on ``threads`` cores."""

    def __init__(self, span: int = 1 << 20, threads: int = 1, region_bytes: Optional[int] = None):
        h = ctypes.c_void_p()
        _check(load().dpgz_par_new(int(span), int(threads), ctypes.byref(h)), "gzip parallel inflate")
        self._h = h
        if region_bytes:
            _check(load().dpgz_par_set_region(h, int(region_bytes)), "gzip parallel inflate")

    def feed(self, data, final: bool = False) -> None:
        keep = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
        _check(load().dpgz_par_feed(self._h, keep.ctypes.data, len(data), int(final)), "gzip stream")

    def read_into(self, out: np.ndarray, off: int, cap: int) -> int:
        """Copy up to ``cap`` inflated bytes to out[off:]; returns how many."""
        n = ctypes.c_uint64(0)
        _check(load().dpgz_par_read(self._h, out.ctypes.data + off, int(cap), ctypes.byref(n)), "gzip stream")
        return int(n.value)

    def stats(self) -> dict:
        st = (ctypes.c_uint64 * 14)()
        _check(load().dpgz_par_state(self._h, st), "gzip stream")
        keys = ("consumed", "produced", "members", "unread", "points", "window_bytes", "ended", "batches",
                "rejected", "ns_find", "ns_decode", "ns_windows", "ns_resolve", "ns_inorder")
        return dict(zip(keys, (int(x) for x in st)))

    def take(self, out_limit: int):
        """(points with out_byte <= out_limit as POINTEX_DTYPE, their windows as bytes)."""
        st = self.stats()
        npts, nwin = st["points"], st["window_bytes"]
        pts = np.zeros(max(1, npts), POINTEX_DTYPE)
        win = np.zeros(max(1, nwin), np.uint8)
        n, w = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _check(load().dpgz_par_take(self._h, int(out_limit), pts.ctypes.data, npts, win.ctypes.data, nwin,
                                    ctypes.byref(n), ctypes.byref(w)), "gzip stream")
        return pts[: int(n.value)], win[: int(w.value)].tobytes()

    def close(self):
        if self._h:
            load().dpgz_par_free(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def is_bgzf(head) -> bool:
    """The first member carries its compressed size (BGZF "BC" extra subfield)."""
    h = bytes(head[:64])
    if len(h) < 18 or h[0] != 0x1F or h[1] != 0x8B or h[2] != 8 or not h[3] & 4:
        return False
    xlen = h[10] | (h[11] << 8)
    q = 12
    while q + 4 <= min(len(h), 12 + xlen):
        slen = h[q + 2] | (h[q + 3] << 8)
        if h[q:q + 2] == b"BC" and slen == 2:
            return True
        q += 4 + slen
    return False


def bgzf_scan(buf: np.ndarray):
    """Complete BGZF members at the start of ``buf``: (in_off, in_len, out_len) uint64 arrays, bytes used."""
    cap = len(buf) // 18 + 1
    a, b, c = (np.zeros(cap, np.uint64) for _ in range(3))
    n, used = ctypes.c_uint64(0), ctypes.c_uint64(0)
    _check(load().dpgz_bgzf_scan(buf.ctypes.data if len(buf) else None, len(buf), a.ctypes.data_as(_U64P),
                                 b.ctypes.data_as(_U64P), c.ctypes.data_as(_U64P), cap, ctypes.byref(n),
                                 ctypes.byref(used)), "BGZF member table")
    k = int(n.value)
    return a[:k], b[:k], c[:k], int(used.value)


def inflate_members(buf: np.ndarray, in_off, in_len, out_off, out_len, out_addr: int, threads: int) -> None:
    """Inflate BGZF members of ``buf`` independently on ``threads`` threads, member i to out_addr + out_off[i]."""
    arrs = [np.ascontiguousarray(x, np.uint64) for x in (in_off, in_len, out_off, out_len)]
    _check(load().dpgz_inflate_members(buf.ctypes.data, *[x.ctypes.data_as(_U64P) for x in arrs], len(arrs[0]),
                                       out_addr, int(threads)), "BGZF inflate")
