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


_lib = None
_ERRORS = {1: "invalid argument", 2: "out of memory", 3: "corrupt gzip/deflate data", 4: "truncated gzip stream"}


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


def inflate_from(points: np.ndarray, i: int, window: bytes, fetch: Callable[[int], Iterable[bytes]]) -> Iterator[bytes]:
    """Inflated bytes from access point ``i`` to the end of the object.

    ``fetch(offset)`` yields the compressed object's bytes from ``offset`` onwards (chunks of any size;
    the caller may stop iterating any time).  Member ends inside a shifted stream are not byte-
    addressable, so at the end of a member the stream continues at the next member-start point."""
    while i < len(points):
        p = points[i]
        member = bool(p["member_start"])
        if member:
            d = zlib.decompressobj(wbits=31)
            src = fetch(int(p["in_byte"]))
            sh = None
        else:
            b = int(p["bits"])
            d = zlib.decompressobj(wbits=-15, zdict=window) if window else zlib.decompressobj(wbits=-15)
            src = fetch(int(p["in_byte"]) - (1 if b else 0))
            sh = _Shifter(b)
        for c in src:
            if sh is not None:
                c = sh.feed(c)
            out = d.decompress(c)
            if out:
                yield out
            if d.eof:
                break
        else:
            if sh is not None and not d.eof:
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
