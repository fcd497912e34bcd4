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
    assert lib.dp_abi_version() == _lib.ABI_VERSION == 2
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


def _header_text():
    return open(os.path.join(REPO, "include", "dpscan.h")).read()


def test_every_out_mode_is_documented():
    """dp_delim_ranges_async's out_mode values the library accepts (0-4) are each described in the header."""
    doc = _header_text()
    src = open(os.path.join(REPO, "dataplug_amd", "csrc", "dpscan.hip")).read()
    assert "out_mode < 0 || out_mode > 4" in src                  # what the library accepts
    for m in ("out_mode 0: uint32", "1: uint64", "2: uint32 low words", "out_mode 3: uint16 low words",
              "out_mode 4: uint8 low bytes"):
        assert m in doc, m
    assert "(2 * cap + 15) & ~15" in doc and "(cap + 15) & ~15" in doc
    assert "(item * cap + 15) & ~15ull" in src and "(tab_off + 8 * ntab + 15) & ~15ull" in src
    assert "congruent mod 16" in doc


@pytest.mark.parametrize("first,last,cap", [(0, 1 << 20, 1000), (70_000, 200_001, 17), (65_536, 65_537, 1),
                                            (5, 5, 0), ((1 << 32) + 3, (1 << 32) + (9 << 16), 12_345)])
def test_out_mode4_layout_matches_header(first, last, cap):
    """The block-table and 256-byte-table offsets and sizes the header documents equal what ScanContext allocates and
    reads for out_mode 4."""
    import numpy as np
    from dataplug_amd.scan.device import ScanContext
    ranges = np.array([first, (first + last) // 2, (first + last) // 2, last], np.uint64)
    j0 = first >> 16
    J = ((last - 1) >> 16) - j0 + 1 if last > first else 1
    s0 = first >> 8
    S = ((last - 1) >> 8) - s0 + 1 if last > first else 1
    tab_off = (cap + 15) & ~15
    sub_off = (tab_off + 8 * J + 15) & ~15
    assert ScanContext.block_table_size(ranges) == (j0, J) and ScanContext.sub_table_size(ranges) == (s0, S)
    assert ScanContext._tab_off(cap, 4) == tab_off and ScanContext._sub_off(cap, ranges) == sub_off
    assert ScanContext.out_bytes(cap, 4, ranges) >= sub_off + 2 * S


@pytest.mark.parametrize("first,last,cap", [(0, 1 << 20, 1000), (70_000, 200_001, 17), (65_536, 65_537, 1),
                                            (5, 5, 0), ((1 << 32) + 3, (1 << 32) + (9 << 16), 12_345)])
def test_out_mode3_layout_matches_header(first, last, cap):
    """The block-table offset and size the header documents equal what ScanContext allocates and reads."""
    import numpy as np
    from dataplug_amd.scan.device import ScanContext
    ranges = np.array([first, (first + last) // 2, (first + last) // 2, last], np.uint64)
    j0 = first >> 16
    J = ((last - 1) >> 16) - j0 + 1 if last > first else 1
    tab_off = (2 * cap + 15) & ~15
    assert ScanContext.block_table_size(ranges) == (j0, J)
    assert ScanContext.out_bytes(cap, 3, ranges) >= tab_off + 8 * J
