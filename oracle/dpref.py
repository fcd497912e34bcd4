"""ctypes binding of oracle/build/libdpref.so — CPU ORACLE, test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "build", "libdpref.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        _lib = ctypes.CDLL(_LIB)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        _lib.dpref_fasta.restype = ctypes.c_int64
        _lib.dpref_fasta.argtypes = [ctypes.c_void_p, ctypes.c_uint64, u64p, ctypes.c_uint64, u64p, ctypes.c_uint64]
        _lib.dpref_delim.restype = ctypes.c_int64
        _lib.dpref_delim.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_uint32, u64p, ctypes.c_uint64, u64p]
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def fasta_pairs(data: np.ndarray, chunks) -> np.ndarray:
    """(n, 2) uint64 (start, end) pairs for a chunk list over the whole object ``data`` (uint8)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    ch = np.ascontiguousarray(np.asarray(chunks, dtype=np.uint64).reshape(-1))
    cap = max(16, len(data) // 512)
    while True:
        out = np.empty(2 * cap, np.uint64)
        n = lib().dpref_fasta(data.ctypes.data, len(data), _ptr(ch), len(ch) // 2, _ptr(out), cap)
        if n <= cap:
            return out[:2 * n].reshape(-1, 2)
        cap = n


def delim(data: np.ndarray, begin: int, end: int, delim: int = 10, every_k: int = 1, emit_add: int = 0):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    cap = max(16, (end - begin) // 16)
    nd = np.zeros(1, np.uint64)
    while True:
        out = np.empty(cap, np.uint64)
        n = lib().dpref_delim(data.ctypes.data, begin, end, delim, every_k, emit_add, _ptr(out), cap, _ptr(nd))
        if n <= cap:
            return out[:n], int(nd[0])
        cap = n
