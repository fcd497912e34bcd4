"""BASELINE-size cases through the C ABI (device-resident), checked exactly.

* 4 GiB synthetic FASTA, chunk_size = size/4 (BASELINE configs[1]) and size/64: every pair vs the C oracle.
* 4.5 GiB FASTA: the uint32 index raises OverflowError like the reference; the uint64 index is exact.
* 8 GiB CSV (configs[2] shape, scaled to keep the host check cheap): the input repeats a base block, so
  the expected newline index is the base block's offsets shifted by every copy — checked in full, plus
  every-4th (FASTQ read ends) on the same bytes.
"""
import math

import numpy as np
import pytest

from dataplug_amd import synth

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
GiB = 1 << 30


def _plan(size, cs):
    n = size // cs
    return [(i * cs, size if cs == n - 1 else (i + 1) * cs) for i in range(n)]


@pytest.fixture(scope="module")
def fasta4(ctx):
    host = synth.tiled_fasta_host(4 * GiB, seed=1)
    d = ctx.workspace("full_in", len(host) + 64)
    ctx.h2d(d.ptr, host)
    return host, d


@pytest.mark.parametrize("div", [4, 64])
def test_fasta_4gib_exact(ctx, fasta4, div):
    from oracle import dpref
    host, d = fasta4
    size = len(host)
    plan = _plan(size, math.ceil(size / div))
    pairs, pending, cend = ctx.fasta_index(d.ptr, size, 0, size, plan, u64=False, cap=size // 512)
    assert (pending < 0).all()
    exp = dpref.fasta_pairs(host, plan)
    assert len(pairs) == len(exp) > 2_000_000
    assert np.array_equal(pairs.astype(np.uint64), exp)
    assert cend[-1] == len(exp)


def test_fasta_over_4gib_overflow_and_u64(ctx):
    from oracle import dpref
    size = 4 * GiB + GiB // 2
    host = synth.tiled_fasta_host(size, seed=2)
    d = ctx.workspace("full_in", size + 64)
    ctx.h2d(d.ptr, host)
    plan = _plan(size, math.ceil(size / 4))
    with pytest.raises(OverflowError):
        ctx.fasta_index(d.ptr, size, 0, size, plan, u64=False, cap=size // 512)
    pairs, pending, _ = ctx.fasta_index(d.ptr, size, 0, size, plan, u64=True, cap=size // 512)
    exp = dpref.fasta_pairs(host, plan)
    assert np.array_equal(pairs, exp)
    assert int(pairs[-1, 1]) > 2**32


def test_csv_8gib_newline_index(ctx):
    base = synth.csv(64 * (1 << 20) - 333, 9)       # ends with '\n'
    size = 8 * GiB
    host = synth.tiled_host(base, size)
    d = ctx.workspace("full_in", size + 64)
    ctx.h2d(d.ptr, host)
    del host
    bnl = np.flatnonzero(base == 10).astype(np.uint64)
    parts = []
    for off, n in synth.tile_plan(len(base), size):
        parts.append(bnl[bnl < n] + np.uint64(off))
    exp = np.concatenate(parts)
    got, nd = ctx.delim_index(d.ptr, size, 0, 0, size, delim=10, u64=True)
    assert nd == len(exp) and np.array_equal(got, exp)
    del got
    got4, nd4 = ctx.delim_index(d.ptr, size, 0, 0, size, delim=10, every_k=4, emit_add=1, u64=True)
    assert nd4 == len(exp) and np.array_equal(got4, exp[3::4] + np.uint64(1))


def test_header_cut_by_chunk_end_far_before_buffer_end(ctx):
    """A header line cut by a chunk end more than 2 GiB before the end of the device buffer: its end comes
    from the resolve kernel's search, whose lane window once truncated (end - pos) to 32 bits and skipped to
    the first '\\n' 2 GiB before the buffer end (found by bench.py's 4 x 4 GiB split).  Every chunk end of
    the plan cuts a header here, and dp_find_delim is checked from the same positions."""
    from oracle import dpref
    size = 2 * GiB + (96 << 20)
    host = synth.tiled_fasta_host(size, seed=5)
    d = ctx.workspace("full_in", size + 64)
    ctx.h2d(d.ptr, host)
    gts = np.flatnonzero(host[: 8 << 20] == ord(">"))
    cuts = [int(p) + 7 for p in gts[[3, 40, 41, 900]]]          # 7 bytes into header lines
    plan = [(0, cuts[0])] + list(zip(cuts[:-1], cuts[1:])) + [(cuts[-1], size)]
    pairs, pending, _ = ctx.fasta_index(d.ptr, size, 0, size, plan, u64=True)
    assert (pending < 0).all()
    exp = dpref.fasta_pairs(host, plan)
    assert np.array_equal(pairs, exp)
    for c in cuts:
        nl = int(np.flatnonzero(host[c:c + 4096] == 10)[0]) + c
        assert ctx.find_delim(d.ptr, size, 0, c, 10) == nl


def _check_delims(ctx, obj, lo, hi, d_ptr, stage):
    """Newline index of object bytes [lo, hi) (uploaded 4 GiB at a time) against the TiledText analytic
    offsets: every offset compared."""
    step = 4 * GiB
    for p in range(lo, hi, step):
        q = min(hi, p + step)
        ctx.h2d(d_ptr + (p - lo), obj.bytes_range(p, q, out=stage))
    got, nd = ctx.delim_index(d_ptr, hi - lo, lo, lo, hi, delim=10, u64=True, cap=obj.count_range(lo, hi) + 64)
    i = 0
    for piece in obj.delims_range(lo, hi):
        assert np.array_equal(got[i:i + len(piece)], piece), (lo, hi, i)
        i += len(piece)
    assert i == len(got) == nd
    return nd


@pytest.mark.parametrize("out_mode", [4, 3])
def test_csv_32gib_configs2_every_offset(ctx, out_mode):
    """BASELINE configs[2]: the newline index of a 32 GiB cities.csv-shaped object in one launch, in a stored
    form (out_mode 4, the default u8s: uint8 low bytes + 256-byte counts + 64 KiB block table; out_mode 3, u16b:
    uint16 low words + the block table); every one of its ~963 M offsets, rebuilt from them, compared with the
    object's analytic newline positions."""
    from dataplug_amd.scan.objects import sub_counts
    size = 32 * GiB
    obj = synth.tiled_csv(size, seed=9)
    d = ctx.workspace("full_in", size + 64)
    stage = np.empty(4 * GiB, np.uint8)
    for p in range(0, size, 4 * GiB):
        ctx.h2d(d.ptr + p, obj.bytes_range(p, min(size, p + 4 * GiB), out=stage))
    del stage
    n_exp = obj.count_range(0, size)
    r = ctx.delim_ranges(d.ptr, size, 0, [(0, size)], out_mode=out_mode, cap=n_exp + 64)
    low, nd, tab = r[0], r[1], r[3]
    assert nd == len(low) == n_exp > 900_000_000
    if out_mode == 4:
        c = sub_counts(r[4], tab, 0, 0)              # entries before every 256-byte boundary
        assert c[0] == 0 and (np.diff(c) >= 0).all() and c[-1] <= n_exp
        unit = np.repeat(np.arange(len(c), dtype=np.uint32), np.diff(np.append(c, np.uint64(n_exp))).astype(np.int64))
        shift = np.uint64(8)
    else:
        unit = None
        shift = np.uint64(16)
    i = 0
    for piece in obj.delims_range(0, size):
        if unit is not None:
            u = unit[i:i + len(piece)].astype(np.uint64)
        else:
            idx = np.arange(i, i + len(piece), dtype=np.int64)
            u = np.searchsorted(tab.astype(np.int64), idx, side="right").astype(np.uint64) - np.uint64(1)
        assert np.array_equal((u << shift) | low[i:i + len(piece)].astype(np.uint64), piece), i
        i += len(piece)
    assert i == nd


def test_vcf_64gib_configs3_eight_parts():
    """BASELINE configs[3]: one 64 GiB VCF whose body [body_offset, size) is cut by the product's part split
    (scan.objects.line_parts) into 8 parts, one worker thread and context per part as
    DATAPLUG_AMD_DEVICES=0,0,0,0,0,0,0,0 runs them; every offset of every part exact, and the parts'
    indexes concatenate to the whole body's."""
    import concurrent.futures as cf
    from dataplug_amd.scan import ScanContext
    from dataplug_amd.scan.objects import line_parts
    size = 64 * GiB
    obj = synth.tiled_vcf(size, seed=9)
    parts = line_parts(len(obj.head), size, 8)
    assert len(parts) == 8 and parts[0][0] == len(obj.head) and parts[-1][1] == size
    assert all(parts[i][1] == parts[i + 1][0] for i in range(7))

    def run(k):
        lo, hi = parts[k]
        c = ScanContext(0)
        try:
            d = c.workspace("in", hi - lo + 64)
            return _check_delims(c, obj, lo, hi, d.ptr, np.empty(min(4 * GiB, hi - lo), np.uint8))
        finally:
            c.close()

    with cf.ThreadPoolExecutor(4) as ex:            # 4 in flight: bounds host staging at 16 GiB
        counts = list(ex.map(run, range(8)))
    assert sum(counts) == obj.count_range(len(obj.head), size) > 800_000_000


class _SynthStore:
    """A read-only storage client over a ``synth.TiledText`` (ranged GETs generate the bytes): the product's
    storage -> pinned -> HBM path without holding the object in host memory."""

    def __init__(self, obj):
        self.obj = obj

    def get_object(self, Bucket, Key, Range=None):
        import io
        a, b = (int(x) for x in Range.split("=")[1].split("-"))
        return {"Body": io.BytesIO(self.obj.bytes_range(a, min(b + 1, self.obj.size)).tobytes())}


def test_vcf_64gib_configs3_stored_u8s_through_product(monkeypatch):
    """verdict r5 #3: configs[3] through the product path in the stored form: ``line_index_object(fmt="u8s")``
    fetches the 64 GiB VCF body by ranged GETs into pinned memory and HBM, cuts it into 8 parts (four device entries,
    two parts each, as eight GPUs would take one each), scans each in out_mode 4 and merges the parts' low bytes,
    256-byte counts and block tables; every one of the ~859 M offsets decoded from the merged tables equals the
    object's analytic newline positions."""
    from types import SimpleNamespace
    from dataplug_amd.scan.objects import ByteOffsets, line_index_object, line_parts, release_workers, sub_counts
    size = 64 * GiB
    obj = synth.tiled_vcf(size, seed=9)
    begin = len(obj.head)
    monkeypatch.setenv("DATAPLUG_AMD_DEVICES", "0,0,0,0")
    assert len(line_parts(begin, size, 4, part_bytes=8 * GiB)) == 8
    co = SimpleNamespace(storage=_SynthStore(obj), path=SimpleNamespace(bucket="b", key="k.vcf"), size=size)
    try:
        bo = line_index_object(co, begin=begin, fmt="u8s", part_bytes=8 * GiB)
    finally:
        release_workers()                         # the four workers' 8 GiB pinned stages and HBM inputs
    assert isinstance(bo, ByteOffsets) and bo.s0 == begin >> 8 and bo.j0 == begin >> 16
    n_exp = obj.count_range(begin, size)
    assert len(bo) == n_exp > 800_000_000
    c = sub_counts(bo.sub, bo.table, bo.s0, bo.j0)
    assert c[0] == 0 and (np.diff(c) >= 0).all() and c[-1] <= n_exp
    unit = np.repeat(np.arange(len(c), dtype=np.uint32), np.diff(np.append(c, np.uint64(n_exp))).astype(np.int64))
    del c
    i = 0
    for piece in obj.delims_range(begin, size):
        u = unit[i:i + len(piece)].astype(np.uint64) + np.uint64(bo.s0)
        assert np.array_equal((u << np.uint64(8)) | bo.low[i:i + len(piece)].astype(np.uint64), piece), i
        i += len(piece)
    assert i == n_exp
