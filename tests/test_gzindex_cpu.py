"""The streamed gzip index pipeline (scan/gzindex.py) on CPU: the inflater thread, piece hand-off, carried
newline ordinals, access points with their windows and line numbers, BGZF member-parallel inflate.

The device side is replaced by a stand-in context whose newline scan is the oracle (oracle/cpu_ref) — this
checks the host pipeline only; tests/test_gpu_dropin.py runs the same pipeline through libdpscan on the GPU.
Expected values come from inflating the whole object at once (gzip.decompress, libdpgz dpgz_build)."""
import gzip
import io

import numpy as np
import pytest

from dataplug_amd import gz, synth
from dataplug_amd.scan import gzindex
from dataplug_amd.scan._lib import DPCapacityError
from oracle import cpu_ref


class _Buf:
    def __init__(self, n):
        self.array = np.zeros(max(16, n), np.uint8)
        self.ptr = self.array.ctypes.data
        self.nbytes = n


class OracleCtx:
    """The few ScanContext calls gzindex makes; the scan is cpu_ref.delim_index over the 'device' bytes."""

    def __init__(self, enforce_cap=False):
        self.mem = {}
        self.out = None
        self.enforce_cap = enforce_cap
        self.cap = None

    def pinned(self, name, n):
        b = _Buf(n)
        self.mem[b.ptr] = b.array
        return b

    def workspace(self, name, n):
        return self.pinned(name, n)

    def _at(self, ptr):
        for base, arr in self.mem.items():
            if base <= ptr < base + len(arr):
                return arr, ptr - base
        raise KeyError(ptr)

    def h2d_async(self, dst, src, n):
        d, i = self._at(dst)
        s, j = self._at(src)
        d[i:i + n] = s[j:j + n]

    def delim_ranges_async(self, d_buf, buf_len, buf_base, ranges, delim, k, add, carry, d_out, mode, cap):
        a, i = self._at(d_buf)
        data = a[i:i + buf_len]
        pos = cpu_ref.delim_index(data, 0, buf_len, delim) + np.uint64(buf_base)
        g = np.arange(len(pos), dtype=np.int64) + carry
        sel = pos[(g % k) == k - 1] + np.uint64(add)
        self.out = (sel, len(pos))
        self.cap = cap
        if self.enforce_cap:                      # the device writes at most cap entries (DP_ERR_CAPACITY)
            d, j = self._at(d_out)
            assert j + 8 * cap <= len(d), "output buffer smaller than its capacity"

    def delim_ranges_result(self, nranges):
        sel, nd = self.out
        if self.enforce_cap and len(sel) > self.cap:
            e = DPCapacityError(3, f"output capacity below {len(sel)} entries")
            e.needed = len(sel)
            raise e
        return len(sel), nd, np.array([nd], np.uint64)

    def d2h(self, out, src):
        out[:] = self.out[0][:len(out)]
        return out


def _reader(blob, step):
    f = io.BytesIO(blob)
    return lambda n: f.read(min(n, step))


def _check(ix, raw: bytes, blob: bytes, k: int, span: int, bgzf: bool):
    a = np.frombuffer(raw, np.uint8)
    nl = np.flatnonzero(a == 10).astype(np.uint64)
    ends = np.frombuffer(ix.ends.read(), "<u8")
    assert np.array_equal(ends, nl[k - 1::k] + np.uint64(1))
    assert ix.newlines == len(nl) and ix.num_records == len(ends) and ix.uncompressed_size == len(raw)
    assert ix.total_lines == len(nl) + (1 if len(raw) and raw[-1:] != b"\n" else 0)
    windows = ix.windows.read()
    assert ix.bgzf == bgzf
    if not bgzf:
        _, pts = gz.build_index(blob, span=span)
        assert len(ix.rows) == len(pts)
        assert [r[1] for r in ix.rows] == pts["in_byte"].tolist()
        assert [r[2] for r in ix.rows] == pts["out_byte"].tolist()
        assert [r[6] for r in ix.rows] == pts["bits"].tolist()
        assert [r[7] for r in ix.rows] == pts["member_start"].tolist()
    member_out = [r[2] for r in ix.rows if r[7]]
    for r in ix.rows:
        ob, wl, wo = r[2], r[4], r[5]
        assert r[3] == int(np.searchsorted(nl, np.uint64(ob))) + 1            # 1-based line holding byte ob
        assert r[8] == int(ob == 0 or raw[ob - 1] == 10)
        if r[7]:
            assert wl == 0
        else:                                                                  # the member's own history
            m0 = max(x for x in member_out if x <= ob)
            assert windows[wo:wo + wl] == raw[max(m0, ob - 32768):ob]
    return ends


def _multi(raw):
    return gzip.compress(raw[:1_234_567], 6) + gzip.compress(raw[1_234_567:2_000_001], 1) + \
        gzip.compress(raw[2_000_001:], 9) + b"\0" * 5


@pytest.mark.parametrize("piece", [1 << 16, 300_007, 64 << 20])
@pytest.mark.parametrize("k", [4, 1, 3])
def test_stream_pieces_match_whole(piece, k):
    raw = synth.fastq(12_000, seed=3).tobytes()
    blob = _multi(raw)
    ix = gzindex.index_stream(OracleCtx(), _reader(blob, 77_777), record_lines=k, span=1 << 16, piece_bytes=piece)
    assert ix.members == 3 and ix.pieces >= len(raw) // piece
    _check(ix, raw, blob, k, 1 << 16, bgzf=False)


@pytest.mark.parametrize("threads,region", [(1, None), (4, 4096), (8, 1 << 14)])
@pytest.mark.parametrize("piece", [1 << 16, 777_777])
def test_parallel_inflate_pieces(threads, region, piece):
    """The same multi-member stream through zlib on one core and the parallel inflater with small
    speculative regions: identical read ends, window rows and windows, across piece boundaries."""
    raw = synth.fastq(12_000, seed=3).tobytes()
    blob = _multi(raw)
    ix = gzindex.index_stream(OracleCtx(), _reader(blob, 55_555), record_lines=4, span=1 << 15, piece_bytes=piece,
                              threads=threads, region_bytes=region)
    assert ix.members == 3
    _check(ix, raw, blob, 4, 1 << 15, bgzf=False)


@pytest.mark.parametrize("piece", [1 << 17, 1_000_003])
def test_bgzf_member_parallel(piece):
    raw = synth.fastq(15_000, seed=7).tobytes()
    blob = synth.bgzf(raw, block=65_280)
    ix = gzindex.index_stream(OracleCtx(), _reader(blob, 1 << 20), span=1 << 18, piece_bytes=piece, threads=4)
    assert ix.bgzf and ix.members == -(-len(raw) // 65_280) + 1
    _check(ix, raw, blob, 4, 1 << 18, bgzf=True)
    starts = [r[2] for r in ix.rows]
    assert starts[0] == 0 and all(b - a >= 1 << 18 for a, b in zip(starts, starts[1:]))


def test_unterminated_last_line_and_empty():
    raw = synth.fastq(500, seed=1).tobytes()[:-1]
    blob = gzip.compress(raw)
    ix = gzindex.index_stream(OracleCtx(), _reader(blob, 1000), piece_bytes=4096)
    _check(ix, raw, blob, 4, 4 << 20, bgzf=False)
    ix = gzindex.index_stream(OracleCtx(), _reader(gzip.compress(b""), 1000))
    assert ix.total_lines == 0 and ix.uncompressed_size == 0 and ix.num_records == 0


def test_corrupt_and_truncated_raise():
    blob = gzip.compress(synth.fastq(2000, seed=2).tobytes())
    with pytest.raises(ValueError):
        gzindex.index_stream(OracleCtx(), _reader(blob[: len(blob) // 2], 1000), piece_bytes=1 << 16)
    bad = bytearray(blob)
    bad[100:140] = b"\xff" * 40
    with pytest.raises(ValueError):
        gzindex.index_stream(OracleCtx(), _reader(bytes(bad), 1000), piece_bytes=1 << 16)
    bg = synth.bgzf(synth.fastq(2000, seed=2).tobytes())
    with pytest.raises(ValueError):
        gzindex.index_stream(OracleCtx(), _reader(bg[:-100], 1 << 20), piece_bytes=1 << 16)


@pytest.mark.parametrize("kind", ["multi", "bgzf"])
def test_preprocess_gzip_then_read_batches(monkeypatch, kind):
    """co.preprocess() of a FASTQ.gz through the streamed pipeline (scan stand-in), then the reference's read
    batching resumes inflating at the stored access points: every line once, in order."""
    from dataplug_amd.cloudobject import CloudObject
    from dataplug_amd.formats.compressed import gzipped as fgz
    from dataplug_amd.formats.genomics import fastq as ffq
    from dataplug_amd.storage import MemoryStore
    monkeypatch.setattr(fgz, "get_context", lambda dev=0: OracleCtx())
    monkeypatch.setenv("DATAPLUG_AMD_DEVICES", "0")
    raw = synth.fastq(20_000, seed=5).tobytes()
    blob = _multi(raw) if kind == "multi" else synth.bgzf(raw)
    name = f"pp_{kind}.fq.gz"
    MemoryStore._named.pop(name, None)
    cfg = {"endpoint_url": f"memory://{name}"}
    co = CloudObject.from_s3(ffq.FASTQGZip, f"s3://b/{name}", fetch=False, s3_config=cfg)
    co.storage.create_bucket(Bucket="b")
    co.storage.put_object(Body=blob, Bucket="b", Key=name)
    co = CloudObject.from_s3(ffq.FASTQGZip, f"s3://b/{name}", s3_config=cfg)
    co.preprocess(extra_args={"span": 1 << 16, "piece_bytes": 200_003})
    lines = [x.decode() for x in raw.split(b"\n")[:-1]]
    assert co.attributes.total_lines == len(lines) and co.attributes.bgzf == (kind == "bgzf")
    ends = ffq.load_read_index(co)
    nl = np.flatnonzero(np.frombuffer(raw, np.uint8) == 10)
    assert np.array_equal(ends, nl[3::4] + 1)
    for nb in (1, 7, 33):
        got = [ln for b in co.partition(ffq.partition_reads_batches, num_batches=nb) for ln in b.get()]
        assert got == lines


@pytest.mark.parametrize("k", [1, 4])
def test_piece_of_empty_lines_fits_the_read_end_capacity(k):
    """A piece that is almost all newlines (FASTQ with empty sequence lines, or blank text lines) has one
    read end per k bytes: the device output is sized for that bound, checked by a stand-in
    that enforces the capacity the pipeline passes, as the device does."""
    raw = (b"@\n\n+\n\n" * 3000) + b"\n" * 20000 + synth.fastq(200, seed=2).tobytes()
    blob = gzip.compress(raw)
    ctx = OracleCtx(enforce_cap=True)
    ix = gzindex.index_stream(ctx, _reader(blob, 4096), record_lines=k, span=1 << 15, piece_bytes=1 << 14,
                              threads=1)
    _check(ix, raw, blob, k, 1 << 15, bgzf=False)


def test_bgzf_long_zero_padding_does_not_spin():
    """More than a batch of zero padding between BGZF members: the padding is dropped and the stream read
    on (it used to rescan the same buffer forever)."""
    raw = synth.fastq(2000, seed=5).tobytes()
    half = len(raw) // 2
    blob = synth.bgzf(raw[:half], block=65_280)
    eof_marker = blob[-28:]                      # the empty BGZF member that ends a BGZF file
    blob = blob[:-28] + bytes(gzindex.BGZF_BATCH + 12345) + synth.bgzf(raw[half:], block=65_280)
    assert eof_marker == blob[-28:]
    ix = gzindex.index_stream(OracleCtx(), _reader(blob, 1 << 20), span=1 << 18, piece_bytes=1 << 17, threads=2)
    assert ix.bgzf
    ends = np.frombuffer(ix.ends.read(), "<u8")
    nl = np.flatnonzero(np.frombuffer(raw, np.uint8) == 10).astype(np.uint64)
    assert np.array_equal(ends, nl[3::4] + np.uint64(1))


def test_reader_error_surfaces_from_parallel_inflate():
    """A GET body that fails mid-stream: the error reaches the caller (no hang in the reader thread)."""
    raw = synth.fastq(20_000, seed=9).tobytes()
    blob = gzip.compress(raw)
    f = io.BytesIO(blob)
    calls = [0]

    def read(n):
        calls[0] += 1
        if calls[0] > 2:
            raise ConnectionError("body reset")
        return f.read(min(n, 50_000))

    with pytest.raises(ConnectionError):
        gzindex.index_stream(OracleCtx(), read, span=1 << 15, piece_bytes=1 << 16, threads=4, region_bytes=4096)
