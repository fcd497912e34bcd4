"""The C ABI: libdpscan.so loads and exports every entry point include/dpscan.h declares, and the ctypes
table (dataplug_amd/scan/_lib.py) binds exactly those.  No compute calls (no GPU needed)."""
import ctypes
import os
import re

import pytest

from dataplug_amd.scan import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(REPO, "include", "dpscan.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dp_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_path():
    fns = header_functions()
    for must in ("dp_fasta_index", "dp_delim_index", "dp_find_delim", "dp_ctx_create", "dp_h2d", "dp_sync",
                 "dp_timing_read", "dp_last_error", "dp_device_count"):
        assert must in fns


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"{_lib.LIB_PATH} missing: run __graft_entry__.build()")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_ctypes_table_matches_header():
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == header_functions()


def test_abi_version_and_errors_without_gpu():
    lib = _lib.load()
    assert lib.dp_abi_version() >= 1
    n = ctypes.c_int(-1)
    rc = lib.dp_device_count(ctypes.byref(n))
    assert rc in (0, _lib.DP_ERR_HIP)
    if rc:
        assert lib.dp_last_error()        # a message, not a crash


def test_no_fallback_when_library_missing(monkeypatch):
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libdpscan.so")
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.DPScanUnavailable):
        _lib.load()
