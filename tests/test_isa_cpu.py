"""The installed libdpscan.so is the library the ISA guard passed (dataplug_amd/isa_guard.py: dataflow over the
gfx950 assembly of EVERY kernel — no touched in-flight load destination, no scratch segment), and the guard
itself flags what it must.

``dataplug_amd.build.build()`` compiles with -save-temps, runs the guard on that exact assembly, and installs
the library only if it passes, next to a stamp with the guard's report and the installed file's sha256; the
loader refuses a library without a matching "ok" stamp."""
import json
import os

import pytest

from dataplug_amd import build as B
from dataplug_amd import isa_guard
from dataplug_amd.scan import _lib

SHIPPED = ["scan_kernel<0,0>", "scan_kernel<0,1>", "scan_kernel<1,0>", "scan_kernel<1,1>", "scan_kernel<1,2>",
           "scan_kernel<1,3>", "map_kernel", "fasta_place_kernel<0>", "fasta_place_kernel<1>", "line_kernel<0>",
           "line_kernel<1>", "line_kernel<2>", "line_kernel<3>", "density_probe_kernel", "fasta_resolve_kernel",
           "find_kernel", "stream_kernel", "stream_rw_kernel"]


def _stamp():
    if not os.path.exists(B.OUT):
        pytest.fail(f"{B.OUT} missing: run __graft_entry__.build()")
    with open(B.stamp_path(B.OUT)) as f:
        return json.load(f)


def test_installed_library_passed_the_guard():
    rep = _stamp()
    assert rep["result"] == "ok" and rep["guard_enforced"], rep
    assert rep["so_sha256"] == B.sha256_file(B.OUT), "the stamp belongs to another build of libdpscan.so"
    assert sorted(rep["kernels"]) == sorted(SHIPPED), rep["kernels"]
    assert rep["n_violations"] == 0 and rep["scratch"] == [] and rep["missing_kernels"] == []
    assert _lib.guard_check(B.OUT)["result"] == "ok"


def test_loader_refuses_unguarded_library(tmp_path):
    lib = tmp_path / "libx.so"
    lib.write_bytes(b"\x7fELF not really")
    with pytest.raises(_lib.DPScanUnavailable, match="no ISA-guard stamp"):
        _lib.guard_check(str(lib))
    (tmp_path / "libx.so.isa.json").write_text(json.dumps({"result": "FAIL", "so_sha256": B.sha256_file(str(lib))}))
    with pytest.raises(_lib.DPScanUnavailable, match="FAIL"):
        _lib.guard_check(str(lib))
    (tmp_path / "libx.so.isa.json").write_text(json.dumps({"result": "ok", "so_sha256": "0" * 64}))
    with pytest.raises(_lib.DPScanUnavailable, match="not loaded"):
        _lib.guard_check(str(lib))


_ASM = """\t.text
_ZN12_GLOBAL__N_110map_kernelILi0EEEvNS_7MapArgsEPKmS3_S3_:
\t;;#ASMSTART
\tbuffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen nt
\t;;#ASMEND
\t{use}
\ts_waitcnt vmcnt(0)
\tv_add_u32_e32 v8, v4, v5
\ts_endpgm
.Lfunc_end0:
\t.amdhsa_kernel _ZN12_GLOBAL__N_110map_kernelILi0EEEvNS_7MapArgsEPKmS3_S3_
\t\t.amdhsa_private_segment_fixed_size {scratch}
\t.end_amdhsa_kernel
"""


@pytest.mark.parametrize("use,scratch,ok", [("v_mov_b32_e32 v9, v1", 0, True),     # untouched: fine
                                            ("v_mov_b32_e32 v9, v5", 0, False),    # reads an in-flight dest
                                            ("v_mov_b32_e32 v6, v1", 0, False),    # overwrites one
                                            ("v_mov_b32_e32 v9, v1", 16, False)])  # spills to scratch
def test_guard_flags_violations(tmp_path, use, scratch, ok):
    p = tmp_path / "k.s"
    p.write_text(_ASM.format(use=use, scratch=scratch))
    touches = isa_guard.check(str(p)) != []
    spills = isa_guard.scratch(str(p)) != []
    assert spills == (scratch > 0)
    assert (not touches and not spills) == ok
    assert (isa_guard.verify(str(p))["scratch"] == []) == (scratch == 0)
    assert isa_guard.short_name(isa_guard.kernel_names(str(p))[0]) == "map_kernel<0>"


_ASM_DMA = """\t.text
_ZN12_GLOBAL__N_111line_kernelILi1ELi2EEEvNS_8LineArgsE:
\t;;#ASMSTART
\tbuffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen nt
\t;;#ASMEND
\t;;#ASMSTART
\ts_mov_b32 m0, s8
\tglobal_load_lds_dwordx4 v[8:9], off sc1
\t;;#ASMEND
\ts_waitcnt vmcnt({n})
\tv_add_u32_e32 v10, v4, v5
\ts_endpgm
.Lfunc_end0:
\t.amdhsa_kernel _ZN12_GLOBAL__N_111line_kernelILi1ELi2EEEvNS_8LineArgsE
\t\t.amdhsa_private_segment_fixed_size 0
\t.end_amdhsa_kernel
"""


@pytest.mark.parametrize("n,ok", [(0, True), (1, True), (2, False)])
def test_guard_counts_lds_dma_loads(tmp_path, n, ok):
    """line_kernel's look-back windows are LDS-DMA loads (no VGPR destination) that still take a vmcnt slot in
    issue order: after one, `s_waitcnt vmcnt(1)` retires the older buffer load, `vmcnt(2)` does not."""
    p = tmp_path / "k.s"
    p.write_text(_ASM_DMA.format(n=n))
    assert (isa_guard.check(str(p)) == []) == ok
    assert isa_guard.short_name(isa_guard.kernel_names(str(p))[0]) == "line_kernel<1,2>"


_ASM_WIN = """\t.text
_ZN12_GLOBAL__N_111line_kernelILi2EEEvNS_8LineArgsE:
\t;;#ASMSTART
\ts_mov_b32 m0, s8
\tglobal_load_lds_dwordx4 v[8:9], off sc1
\t;;#ASMEND
\t;;#ASMSTART
\tbuffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen nt
\t;;#ASMEND
\ts_waitcnt vmcnt({n})
\t;;#ASMSTART
\tds_read_b64 v[10:11], v3 ; dp_win_read
\ts_waitcnt lgkmcnt(0)
\t;;#ASMEND
\ts_endpgm
.Lfunc_end0:
\t.amdhsa_kernel _ZN12_GLOBAL__N_111line_kernelILi2EEEvNS_8LineArgsE
\t\t.amdhsa_private_segment_fixed_size 0
\t.end_amdhsa_kernel
"""


@pytest.mark.parametrize("n,ok", [(1, True), (0, True), (2, False)])
def test_guard_flags_a_window_read_before_its_lds_dma(tmp_path, n, ok):
    """a tagged read of line_kernel's look-back window while its LDS-DMA load may still be in flight is a
    violation: with a buffer load issued after the window, `vmcnt(1)` retires the window, `vmcnt(2)` does not."""
    p = tmp_path / "k.s"
    p.write_text(_ASM_WIN.format(n=n))
    assert (isa_guard.check(str(p)) == []) == ok


def test_stamp_matches_the_source_tree():
    """The installed library was built from the kernel source in the tree (a stale build that passed the guard on
    older source does not pass this)."""
    rep = _stamp()
    assert rep.get("src_sha256") == B.sha256_file(B.SRC), "libdpscan.so was built from another dpscan.hip: rebuild"
