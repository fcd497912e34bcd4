"""Partition strategies + slice get() against the REFERENCE's own outputs (tests/golden/*.json).

The index a strategy reads is built here from the object bytes (numpy: the newline positions / the golden
FASTA index are inputs, not the thing under test); what is tested is the host logic that turns an index
into slices — CSV/VCF bodies from the newline index (formats/_lines.py), FASTA slices, FASTQ batches.
Objects: the reference's sample files are rebuilt from the golden single-slice get() and checked against
the recorded sha256; synthetic objects are regenerated from their seeds (dataplug_amd.synth).
"""
import base64
import builtins
import json
import os

import numpy as np
import pytest

from dataplug_amd import synth
from dataplug_amd.cloudobject import CloudObject
from dataplug_amd.entities import get_slices
from dataplug_amd.formats._lines import SliceError, store_line_index
from dataplug_amd.scan.objects import BlockedOffsets, ByteOffsets, PagedOffsets
from dataplug_amd.preprocessing.handler import upload_metadata
from dataplug_amd.preprocessing.metadata import PreprocessingMetadata
from dataplug_amd.storage import MemoryStore

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def _as_format(off: np.ndarray, fmt):
    """The stored index forms built from plain uint64 offsets (what the GPU writes for each)."""
    if fmt in (True, "u32p"):
        return PagedOffsets(off.astype(np.uint32), [])
    if fmt == "u16b":
        j0 = int(off[0]) >> 16 if len(off) else 0
        j1 = int(off[-1]) >> 16 if len(off) else 0
        tab = np.searchsorted(off, np.arange(j0, j1 + 1, dtype=np.uint64) << np.uint64(16)).astype(np.uint64)
        return BlockedOffsets((off & np.uint64(0xFFFF)).astype(np.uint16), tab, j0)
    if fmt == "u8s":
        return byte_offsets(off, int(off[0]) if len(off) else 0, int(off[-1]) + 1 if len(off) else 1)
    return off


def byte_offsets(off: np.ndarray, first: int, last: int) -> ByteOffsets:
    """The uint8 index (out_mode 4) of sorted offsets in [first, last), as the GPU writes it: low bytes, the low 16
    bits of the entries before every 256-byte boundary, the entries before every 64 KiB boundary (boundaries at or
    below ``first`` read as 0)."""
    s0, s1 = first >> 8, (last - 1) >> 8
    j0, j1 = first >> 16, (last - 1) >> 16
    sb = np.arange(s0, s1 + 1, dtype=np.uint64) << np.uint64(8)
    sub = (np.searchsorted(off, sb) & 0xFFFF).astype(np.uint16)
    if first & 0xFF:
        sub[0] = 0
    tab = np.searchsorted(off, np.arange(j0, j1 + 1, dtype=np.uint64) << np.uint64(16)).astype(np.uint64)
    if first & 0xFFFF:
        tab[0] = 0
    return ByteOffsets((off & np.uint64(0xFF)).astype(np.uint8), sub, tab, s0, j0)


def _co(fmt, name: str, data: bytes, attrs: dict, meta: bytes = None, nl=True, begin=0, paged="u16b"):
    store = f"golden_{name}_{fmt.co_class.__name__}"
    MemoryStore._named.pop(store, None)
    co = CloudObject.from_s3(fmt, f"s3://dataplug/{name}", fetch=False, s3_config={"endpoint_url": f"memory://{store}"})
    co.storage.create_bucket(Bucket="dataplug")
    co.storage.create_bucket(Bucket="dataplug.meta")
    co.storage.put_object(Body=data, Bucket="dataplug", Key=name)
    if nl:
        arr = np.frombuffer(data, np.uint8)
        off = np.flatnonzero(arr[begin:] == 10).astype(np.uint64) + np.uint64(begin)
        attrs = dict(attrs, **store_line_index(co, _as_format(off, paged)))
    upload_metadata(co, PreprocessingMetadata(metadata=meta, attributes=attrs))
    co.fetch()
    return co


def _csv_objects():
    for rec in _load("csv_slices.json")["objects"]:
        if rec["object"] == "synth_csv":
            data = bytes(synth.csv(1 << 16, 5))
        elif rec["object"] == "wide_csv":
            data = bytes(synth.csv_wide(1 << 16, 5))
        else:
            data = rec["num_chunks"]["1"][0][2].encode()        # one slice from byte 0 = the whole object
        assert synth.sha256(np.frombuffer(data, np.uint8)) == rec["sha256"]
        yield rec, data


def _ref_error(name):
    """The exception class the golden recorded for the reference's get(): a builtin, or the storage
    ClientError (a ranged GET past the end of the object, InvalidRange on S3)."""
    from dataplug_amd.storage.errors import ClientError
    return {"ClientError": ClientError}.get(name) or getattr(builtins, name)


def _vcf_objects():
    for rec in _load("vcf_slices.json")["objects"]:
        if rec["object"] == "synth_vcf":
            data = bytes(synth.vcf(1 << 16, 6))
        elif rec["object"] == "wide_vcf":
            data = bytes(synth.vcf_wide(1 << 16, 6))
        else:
            one = rec["num_chunks"]["1"][0][2]                  # header meta + "\n" + body
            body = one[len(rec["meta"]) + 1:].encode()
            head = rec["meta"].encode() + b"\n"
            data = head + body
        if synth.sha256(np.frombuffer(data, np.uint8)) != rec["sha256"]:
            pytest.skip(f"{rec['object']}: header not recoverable byte-exactly from the golden meta")
        yield rec, data


@pytest.mark.parametrize("paged", ["u8s", "u16b", "u32p", "u64"])
def test_csv_partitions_match_reference(paged):
    from dataplug_amd.formats.generic import csv as fcsv
    checked = 0
    for rec, data in _csv_objects():
        co = _co(fcsv.CSV, rec["object"], data, {"columns": rec["columns"], "dtypes": rec["dtypes"]}, paged=paged)
        cases = [(fcsv.partition_num_chunks, {"num_chunks": int(n)}, v) for n, v in rec["num_chunks"].items()]
        cases += [(fcsv.partition_chunk_size, {"chunk_size": int(c)}, v) for c, v in rec["chunk_size"].items()]
        for strat, kw, expected in cases:
            slices = co.partition(strat, **kw)
            assert [[s.range_0, s.range_1] for s in slices] == [e[:2] for e in expected], (rec["object"], kw)
            for s, e in zip(slices, expected):
                if isinstance(e[2], dict):
                    with pytest.raises(_ref_error(e[2]["error"])) as ei:   # the reference's class
                        s.get()
                    assert isinstance(ei.value, SliceError)
                else:
                    assert s.get() == e[2], (rec["object"], kw, s.chunk_id)
                checked += 1
            if not any(isinstance(e[2], dict) for e in expected):
                assert get_slices(slices, threads=4) == [e[2] for e in expected]
    assert checked > 100


@pytest.mark.parametrize("paged", ["u8s", "u16b", "u32p", "u64"])
def test_vcf_partitions_match_reference(paged):
    from dataplug_amd.formats.genomics import vcf as fvcf
    for rec, data in _vcf_objects():
        co = _co(fvcf.VCF, rec["object"], data,
                 {"columns": rec["columns"], "vcf_attributes": rec["vcf_attributes"],
                  "body_offset": rec["body_offset"]}, meta=rec["meta"].encode(), begin=rec["body_offset"],
                 paged=paged)
        for n, expected in rec["num_chunks"].items():
            slices = co.partition(fvcf.partition_num_chunks, num_chunks=int(n))
            assert [[s.range_0, s.range_1] for s in slices] == [e[:2] for e in expected]
            for s, e in zip(slices, expected):
                if isinstance(e[2], dict):
                    with pytest.raises(_ref_error(e[2]["error"])) as ei:   # the reference's class
                        s.get()
                    assert isinstance(ei.value, SliceError)
                else:
                    assert s.get() == e[2], (rec["object"], n, s.chunk_id)


def test_vcf_header_parse_matches_reference():
    from dataplug_amd.formats.genomics.vcf import parse_vcf_header
    import io
    for rec, data in _vcf_objects():
        header, meta, columns, bo = parse_vcf_header(io.BytesIO(data))
        assert bo == rec["body_offset"]
        assert columns == rec["columns"]
        assert meta == rec["vcf_attributes"]
        assert "\n".join(header) == rec["meta"]


def _fasta_object(name):
    if name == "sample":
        z = np.load(os.path.join(GOLDEN, "fasta_cases.npz"))
        kinds = list(z["kind"])
        i = kinds.index("sample")
        return bytes(z["data"][z["data_off"][i]:z["data_off"][i + 1]])
    if name == "synth1":
        return bytes(synth.fasta(1 << 18, 11))
    return None


def test_fasta_partitions_match_reference():
    from dataplug_amd.formats.genomics import fasta as ffa
    from oracle import cpu_ref          # checker: builds the index input the strategy reads
    n_checked = 0
    for rec in _load("fasta_slices.json"):
        data = _fasta_object(rec["object"])
        if data is None:
            continue
        idx, nseq = cpu_ref.fasta_index(data, rec["chunk_size"])
        co = _co(ffa.FASTA, rec["object"], data, {"num_sequences": nseq}, meta=idx, nl=False)
        slices = co.partition(ffa.partition_chunks_strategy, num_chunks=rec["num_chunks"])
        got = [[s.offset, None if s.header is None else list(s.header), s.range_0, s.range_1] for s in slices]
        assert got == rec["slices"], (rec["object"], rec["num_chunks"])
        if "get" in rec:
            assert [base64.b64encode(s.get()).decode() for s in slices] == rec["get"]
        assert get_slices(slices, threads=4) == [s.get() for s in slices]
        n_checked += 1
    assert n_checked >= 5


def test_fastq_read_batches_match_reference():
    from dataplug_amd.formats.genomics.fastq import read_pairs
    g = _load("fastq_batches.json")
    for c in g["cases"]:
        assert [list(p) for p in read_pairs(c["total_lines"], c["num_batches"])] == c["line_pairs"]
    with pytest.raises(Exception) as e:
        read_pairs(10, 2)
    assert str(e.value) == g["non_multiple_of_4_error"]


@pytest.mark.parametrize("preload", [True, False])
def test_paged_line_index_across_4gib_pages(monkeypatch, preload):
    """The stored paged form (uint32 low words + entries below each 4 GiB boundary) read back by LineIndex,
    preloaded or block by block over ranged GETs: the same answers as the uint64 offsets."""
    from dataplug_amd.formats import _lines
    from dataplug_amd.scan.objects import BlockedOffsets, PagedOffsets
    if not preload:
        monkeypatch.setattr(_lines, "_PRELOAD_BYTES", 1024)
    rng = np.random.default_rng(3)
    G = 1 << 30
    off = np.unique(rng.integers(3 * G, 17 * G, 50_000).astype(np.uint64))
    pages = [int(np.searchsorted(off, np.uint64(p << 32))) for p in range(1, 5)]   # boundaries 4, 8, 12, 16 GiB
    co = _co(_lines_fmt(), "paged", b"x" * 16, {}, nl=False)
    attrs = store_line_index(co, PagedOffsets(off.astype(np.uint32), pages))
    assert attrs["line_index_dtype"] == "u32p" and attrs["line_index_pages"] == pages
    li = _lines.LineIndex(storage=co.storage, bucket=co.meta_path.bucket, key=attrs["line_index_key"],
                          count=attrs["num_lines"], pages=attrs["line_index_pages"])
    assert np.array_equal(li._fetch(0, li.count), off)
    for x in [0, 3 * G, 4 * G - 1, 4 * G, 4 * G + 1, 8 * G + 12345, 16 * G, 17 * G, int(off[777]), int(off[-1]) + 1]:
        i = int(np.searchsorted(off, np.uint64(x)))
        assert li.nxt(x) == (int(off[i]) + 1 if i < len(off) else None), x
        assert li.contains(x) == (i < len(off) and int(off[i]) == x)


def _lines_fmt():
    from dataplug_amd.formats.generic.csv import CSV
    return CSV


@pytest.mark.parametrize("preload", [True, False])
def test_blocked_line_index_sparse_and_dense_blocks(monkeypatch, preload):
    """uint16 low words + 64 KiB block table, read back by LineIndex (preloaded or block-fetched): empty
    blocks, many entries per block, offsets past 2^32, a first block that starts below the first byte."""
    from dataplug_amd.formats import _lines
    if not preload:
        monkeypatch.setattr(_lines, "_PRELOAD_BYTES", 1024)
    rng = np.random.default_rng(4)
    G = 1 << 30
    dense = rng.integers(5 * G + 123, 5 * G + (1 << 20), 40_000)
    sparse = rng.integers(5 * G + (1 << 20), 7 * G, 3_000)
    off = np.unique(np.concatenate([dense, sparse]).astype(np.uint64))
    bo = _as_format(off, "u16b")
    assert np.array_equal(bo.to_u64(), off)
    co = _co(_lines_fmt(), "blocked", b"x" * 16, {}, nl=False)
    attrs = store_line_index(co, bo)
    assert attrs["line_index_dtype"] == "u16b"
    blocks = np.frombuffer(co.storage.get_object(Bucket=co.meta_path.bucket, Key=attrs["line_index_blocks_key"])
                           ["Body"].read(), "<u8")
    li = _lines.LineIndex(storage=co.storage, bucket=co.meta_path.bucket, key=attrs["line_index_key"],
                          count=attrs["num_lines"], blocks=blocks, block0=attrs["line_index_block0"])
    assert np.array_equal(li._fetch(0, li.count), off)
    for x in [0, 5 * G, 5 * G + 123, 5 * G + 65536, 6 * G, int(off[9999]), int(off[-1]), int(off[-1]) + 1, 8 * G]:
        i = int(np.searchsorted(off, np.uint64(x)))
        assert li.nxt(x) == (int(off[i]) + 1 if i < len(off) else None), x
        assert li.contains(x) == (i < len(off) and int(off[i]) == x)


@pytest.mark.parametrize("preload", [True, False])
@pytest.mark.parametrize("first_delta", [0, 123, 256])
def test_byte_line_index_sparse_and_dense(monkeypatch, preload, first_delta):
    """uint8 low bytes + 256-byte counts + 64 KiB block table (out_mode 4), read back by LineIndex (preloaded, or block
    by block with the 256-byte counts of the blocks they span): 64 KiB blocks of nearly every byte a newline (their
    256-byte counts wrap 16 bits within the index), empty blocks, offsets past 2^32, first bytes on and off 256-byte
    and 64 KiB boundaries."""
    from dataplug_amd.formats import _lines
    if not preload:
        monkeypatch.setattr(_lines, "_PRELOAD_BYTES", 1024)
    rng = np.random.default_rng(5)
    G = 1 << 30
    first = 5 * G + first_delta
    full = np.arange(first + 70_000, first + 70_000 + 65_535 * 3, dtype=np.uint64)        # every byte: dense blocks
    sparse = rng.integers(first + 400_000, 7 * G, 3_000).astype(np.uint64)
    mid = rng.integers(first, first + 70_000, 500).astype(np.uint64)
    off = np.unique(np.concatenate([np.asarray([first], np.uint64), mid, full, sparse]))
    last = int(off[-1]) + 1 + 1000
    bo = byte_offsets(off, first, last)
    assert np.array_equal(bo.to_u64(), off)
    co = _co(_lines_fmt(), "bytes", b"x" * 16, {}, nl=False)
    attrs = store_line_index(co, bo)
    assert attrs["line_index_dtype"] == "u8s"
    blocks = np.frombuffer(co.storage.get_object(Bucket=co.meta_path.bucket, Key=attrs["line_index_blocks_key"])
                           ["Body"].read(), "<u8")
    li = _lines.LineIndex(storage=co.storage, bucket=co.meta_path.bucket, key=attrs["line_index_key"],
                          count=attrs["num_lines"], blocks=blocks, block0=attrs["line_index_block0"],
                          sub_key=attrs["line_index_sub_key"], sub0=attrs["line_index_sub0"])
    assert np.array_equal(li._fetch(0, li.count), off)
    assert np.array_equal(li._fetch(1000, 70_000), off[1000:70_000])
    for x in [0, first, first + 1, first + 70_000, first + 70_000 + 65_535, 6 * G, int(off[9999]), int(off[-1]),
              int(off[-1]) + 1, 8 * G]:
        i = int(np.searchsorted(off, np.uint64(x)))
        assert li.nxt(x) == (int(off[i]) + 1 if i < len(off) else None), x
        assert li.contains(x) == (i < len(off) and int(off[i]) == x)


def test_byte_line_index_sparse_reads_follow_entries(monkeypatch):
    """a sparse uint8 index (1 MB lines over 2 GB) is not preloaded when its 256-byte counts (2 B per
    256 object bytes) exceed the preload budget, and a block of entries reads the counts of the 64 KiB blocks those
    entries lie in, not of every block they span."""
    from dataplug_amd.formats import _lines
    monkeypatch.setattr(_lines, "_PRELOAD_BYTES", 1 << 20)
    rng = np.random.default_rng(11)
    first = (3 << 30) + 77
    off = np.unique((first + np.arange(2_000, dtype=np.int64) * 1_000_003 + rng.integers(0, 4096, 2_000))
                    .astype(np.uint64))
    bo = byte_offsets(off, first, int(off[-1]) + 1)
    co = _co(_lines_fmt(), "sparse_u8s", b"x" * 16, {}, nl=False)
    attrs = store_line_index(co, bo)
    blocks = np.frombuffer(co.storage.get_object(Bucket=co.meta_path.bucket, Key=attrs["line_index_blocks_key"])
                           ["Body"].read(), "<u8")
    fetched = []
    real_get = co.storage.get_object

    def counting_get(**kw):
        res = real_get(**kw)
        if kw.get("Key") == attrs["line_index_sub_key"]:
            body = res["Body"].read()
            fetched.append(len(body))
            res = dict(res, Body=__import__("io").BytesIO(body))
        return res
    monkeypatch.setattr(co.storage, "get_object", counting_get)
    li = _lines.LineIndex(storage=co.storage, bucket=co.meta_path.bucket, key=attrs["line_index_key"],
                          count=attrs["num_lines"], blocks=blocks, block0=attrs["line_index_block0"],
                          sub_key=attrs["line_index_sub_key"], sub0=attrs["line_index_sub0"])
    assert li._arr is None and not fetched                     # 16 MB of counts: not preloaded
    for x in [0, first, int(off[7]), int(off[7]) + 1, int(off[1234]) - 5, int(off[-1]), int(off[-1]) + 1]:
        i = int(np.searchsorted(off, np.uint64(x)))
        assert li.nxt(x) == (int(off[i]) + 1 if i < len(off) else None), x
    assert np.array_equal(li._fetch(0, li.count), off)
    span = 2 * (len(bo.sub))
    # each entry's 64 KiB block: 512 B of counts; two blocks at most per entry (a run never joins blocks > 4 apart)
    assert sum(fetched) <= 2 * (2 * 512 * len(off)) < span / 3, (sum(fetched), span)


def test_auto_index_form_follows_density():
    """``index_format="auto"`` (the CSV / VCF default): u8s while the object holds a newline at least every 128 bytes
    (a sample of 8 ranged GETs of 64 KiB), u16b for sparser objects; small objects are read whole."""
    from dataplug_amd.scan.objects import line_index_form
    rng = np.random.default_rng(3)

    def obj(line_len, size):
        data = rng.integers(65, 90, size, dtype=np.uint8)
        data[line_len - 1::line_len] = 10
        return _co(_lines_fmt(), f"dens{line_len}_{size}", data.tobytes(), {}, nl=False)
    for line_len, size, want in [(36, 8 << 20, "u8s"), (127, 8 << 20, "u8s"), (129, 8 << 20, "u16b"),
                                 (100_000, 8 << 20, "u16b"), (40, 100_000, "u8s"), (5_000, 100_000, "u16b")]:
        co = obj(line_len, size)
        assert line_index_form(co, 0, size) == want, (line_len, size)
    co = obj(36, 1 << 20)
    assert line_index_form(co, 5, 5) == "u8s"


def test_index_put_error_is_the_low_bytes_error(monkeypatch):
    """when the low-bytes PUT and a side PUT both fail, the low bytes' error is raised (the side PUTs are
    waited for, never masking it)."""
    from dataplug_amd.formats import _lines
    off = np.arange(100, 5_000, 37, dtype=np.uint64)
    co = _co(_lines_fmt(), "put_err", b"x" * 16, {}, nl=False)

    def put(**kw):
        raise RuntimeError("low" if kw["Key"].endswith(".lines") else "side")
    monkeypatch.setattr(co.storage, "put_object", put)
    with pytest.raises(RuntimeError, match="^low$"):
        store_line_index(co, byte_offsets(off, 100, 5_000))


def test_index_put_pool_after_fork():
    """a forked child gets a new side-PUT executor (the parent's worker thread does not exist there)."""
    from dataplug_amd.formats import _lines
    assert _lines._put_pool().submit(lambda: 7).result(timeout=10) == 7
    pid = os.fork()
    if pid == 0:                                   # pragma: no cover - the child
        try:
            ok = _lines._put_pool().submit(lambda: 7).result(timeout=10) == 7
        except BaseException:
            ok = False
        os._exit(0 if ok else 1)
    _, status = os.waitpid(pid, 0)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0
