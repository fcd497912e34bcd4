"""ctypes binding of libdpscan.so (the C ABI declared in include/dpscan.h).

The library is built in-tree (``__graft_entry__.build()`` / ``python -m dataplug_amd.build``) into
``dataplug_amd/lib/libdpscan.so``.  There is NO fallback: if the library is missing or cannot be loaded
the import of anything that scans raises ``DPScanUnavailable``.  Nor is a library loaded that the build's
ISA guard did not pass: ``<lib>.isa.json`` (written by ``dataplug_amd.build``) must say "ok" and carry the
sha256 of the very file being loaded (a library whose kernels touch an in-flight load destination can fault
the GPU).
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPSCAN_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libdpscan.so"))

DP_OK = 0
DP_ERR_INVALID = 1
DP_ERR_HIP = 2
DP_ERR_CAPACITY = 3
DP_ERR_OVERFLOW = 4
DP_ERR_TIMEOUT = 5
# dp_ctx_set_form / dp_ctx_get_form settings (include/dpscan.h)
DP_FORM_FASTA = 0
DP_FORM_DELIM = 1
DP_FORM_DELIM_LINE_MAX = 2
DP_FORM_DELIM_DENSE = 3

# (name, restype, argtypes) for every symbol include/dpscan.h declares
_c = ctypes
_p = _c.c_void_p
_u64 = _c.c_uint64
_u64p = _c.POINTER(_c.c_uint64)
_i64p = _c.POINTER(_c.c_int64)
SIGNATURES = [
    ("dp_abi_version", _c.c_int, []),
    ("dp_last_error", _c.c_char_p, []),
    ("dp_device_count", _c.c_int, [_c.POINTER(_c.c_int)]),
    ("dp_ctx_create", _c.c_int, [_c.c_int, _c.POINTER(_p)]),
    ("dp_ctx_destroy", _c.c_int, [_p]),
    ("dp_ctx_get_stream", _c.c_int, [_p, _c.POINTER(_p)]),
    ("dp_ctx_set_stream", _c.c_int, [_p, _p]),
    ("dp_ctx_device", _c.c_int, [_p, _c.POINTER(_c.c_int)]),
    ("dp_ctx_wait", _c.c_int, [_p, _p]),
    ("dp_malloc", _c.c_int, [_p, _u64, _c.POINTER(_p)]),
    ("dp_free", _c.c_int, [_p, _p]),
    ("dp_host_alloc", _c.c_int, [_u64, _c.POINTER(_p)]),
    ("dp_host_free", _c.c_int, [_p]),
    ("dp_h2d", _c.c_int, [_p, _p, _p, _u64]),
    ("dp_d2h", _c.c_int, [_p, _p, _p, _u64]),
    ("dp_sync", _c.c_int, [_p]),
    ("dp_fasta_index", _c.c_int, [_p, _p, _u64, _u64, _u64, _u64p, _u64, _p, _c.c_int, _u64, _u64p, _i64p, _u64p]),
    ("dp_fasta_index_async", _c.c_int, [_p, _p, _u64, _u64, _u64, _u64p, _u64, _p, _c.c_int, _u64]),
    ("dp_fasta_result", _c.c_int, [_p, _u64p, _i64p, _u64p]),
    ("dp_delim_index", _c.c_int, [_p, _p, _u64, _u64, _u64, _u64, _c.c_uint32, _c.c_uint32, _c.c_uint32, _p,
                                  _c.c_int, _u64, _u64p, _u64p]),
    ("dp_delim_index_async", _c.c_int, [_p, _p, _u64, _u64, _u64, _u64, _c.c_uint32, _c.c_uint32, _c.c_uint32,
                                        _p, _c.c_int, _u64]),
    ("dp_delim_result", _c.c_int, [_p, _u64p, _u64p]),
    ("dp_delim_ranges_async", _c.c_int, [_p, _p, _u64, _u64, _u64p, _u64, _c.c_uint32, _c.c_uint32, _c.c_uint32,
                                         _u64, _p, _c.c_int, _u64]),
    ("dp_delim_ranges_result", _c.c_int, [_p, _u64p, _u64p, _u64p]),
    ("dp_find_delim", _c.c_int, [_p, _p, _u64, _u64, _u64, _c.c_uint32, _i64p]),
    ("dp_stream_read", _c.c_int, [_p, _p, _u64, _c.c_int]),
    ("dp_stream_rw", _c.c_int, [_p, _p, _u64, _p, _c.c_uint32, _c.c_int]),
    ("dp_timing_enable", _c.c_int, [_p, _c.c_int]),
    ("dp_timing_read", _c.c_int, [_p, _c.POINTER(_c.c_double), _u64p]),
    ("dp_debug_profile", _c.c_int, [_p, _u64p, _u64, _c.POINTER(_c.c_int), _c.POINTER(_c.c_int)]),
    ("dp_alloc_counts", _c.c_int, [_u64p, _u64p]),
    ("dp_ctx_set_form", _c.c_int, [_p, _c.c_int, _u64]),
    ("dp_ctx_get_form", _c.c_int, [_p, _c.c_int, _u64p]),
    ("dp_scan_delim_form", _c.c_int, [_p, _u64, _c.c_int, _c.POINTER(_c.c_int)]),
    ("dp_last_delim_form", _c.c_int, [_p, _c.POINTER(_c.c_int)]),
    ("dp_scan_geometry", _c.c_int, [_p, _c.POINTER(_c.c_int), _c.POINTER(_c.c_int)]),
]


class DPScanUnavailable(ImportError):
    """libdpscan.so is missing or unloadable: the HIP path cannot run (there is no CPU fallback)."""


class DPScanError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"dpscan error {code}: {msg}")
        self.code = code


class DPCapacityError(DPScanError):
    pass


_lib = None
ABI_VERSION = 2                          # include/dpscan.h DP_ABI_VERSION: the oldest library these signatures fit


def load():
    """Load libdpscan.so once (raises DPScanUnavailable)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DPScanUnavailable(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
                                f"g.build()'` (hipcc --offload-arch=gfx950)")
    guard_check(LIB_PATH)
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the ROCm runtime being present
        raise DPScanUnavailable(f"cannot load {LIB_PATH}: {e}") from e
    lib.dp_abi_version.restype = ctypes.c_int
    ver = int(lib.dp_abi_version())
    if ver < ABI_VERSION and "DPSCAN_LIB" not in os.environ:
        raise DPScanUnavailable(f"{LIB_PATH} has ABI version {ver}, this binding needs {ABI_VERSION} "
                                f"(dp_scan_delim_form's argument list changed in 2): rebuild it")
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name, None)
        if fn is None:
            if "DPSCAN_LIB" in os.environ:     # an older build loaded for a same-box A/B: it lacks newer entry points
                continue
            raise DPScanUnavailable(f"{LIB_PATH} does not export {name}: rebuild it")
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def guard_check(path: str) -> dict:
    """The ISA-guard stamp of ``path`` (raises DPScanUnavailable unless it passed for exactly this file)."""
    stamp = path + ".isa.json"
    try:
        with open(stamp) as f:
            rep = json.load(f)
    except (OSError, ValueError) as e:
        raise DPScanUnavailable(f"{path} has no ISA-guard stamp ({e}): rebuild it with python -m dataplug_amd.build") from e
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    if rep.get("result") != "ok" or rep.get("so_sha256") != h.hexdigest():
        raise DPScanUnavailable(f"{path}: ISA guard {rep.get('result')!r}, stamp for sha256 "
                                f"{str(rep.get('so_sha256'))[:12]}, file {h.hexdigest()[:12]}: not loaded")
    return rep


def check(rc: int) -> None:
    if rc == DP_OK:
        return
    msg = (load().dp_last_error() or b"").decode(errors="replace")
    if rc == DP_ERR_OVERFLOW:
        raise OverflowError(msg or "Python integer out of bounds for uint32")
    if rc == DP_ERR_CAPACITY:
        raise DPCapacityError(rc, msg)
    raise DPScanError(rc, msg)


def alloc_counts():
    """(device allocations, pinned host allocations) libdpscan has made in this process (dp_alloc_counts)."""
    d, h = ctypes.c_uint64(0), ctypes.c_uint64(0)
    check(load().dp_alloc_counts(ctypes.byref(d), ctypes.byref(h)))
    return int(d.value), int(h.value)


def device_count() -> int:
    n = ctypes.c_int(0)
    check(load().dp_device_count(ctypes.byref(n)))
    return int(n.value)
