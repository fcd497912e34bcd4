"""Gzip access points (libdpgz.so + dataplug_amd.gz) and GZipTextSlice resuming mid-object, on CPU.

The window table is built from numpy newline positions here (the GPU scan builds them in
preprocess_gzip; tests/test_gpu_dropin.py runs that path).  Checked: inflating from every access point
(mid-member, non-zero bit offsets, across gzip members, zero padding) reproduces the stream, and the
reference's read batching yields every line exactly once in order."""
import gzip
import io
import os
import zlib

import numpy as np
import pytest

from dataplug_amd import gz, synth
from dataplug_amd.cloudobject import CloudObject
from dataplug_amd.formats.compressed import gzipped as fgz
from dataplug_amd.formats.genomics import fastq as ffq
from dataplug_amd.preprocessing.handler import upload_metadata
from dataplug_amd.preprocessing.metadata import PreprocessingMetadata
from dataplug_amd.storage import MemoryStore


@pytest.fixture(scope="module", autouse=True)
def _built():
    if not os.path.exists(gz.LIB_PATH):
        from dataplug_amd.build import build_gz
        build_gz()


def _raw(n=30000, seed=3):
    return synth.fastq(n, seed).tobytes()


def _multi(raw):
    return gzip.compress(raw[:1_234_567], 6) + gzip.compress(raw[1_234_567:2_000_001], 1) + \
        gzip.compress(raw[2_000_001:], 9) + b"\0" * 5


@pytest.mark.parametrize("span", [1 << 16, 1 << 20])
def test_resume_from_every_point(span):
    raw = _raw()
    blob = _multi(raw)
    out, pts = gz.build_index(blob, span=span)
    assert out.tobytes() == raw
    assert int(pts["member_start"].sum()) == 3
    assert (np.diff(pts["out_byte"].astype(np.int64)) > 0).all()
    assert set(pts["bits"].tolist()) - {0}, "expected points at non-byte-aligned block starts"

    def fetch(off):
        for a in range(off, len(blob), 77_777):
            yield blob[a:a + 77_777]

    for i in range(len(pts)):
        w = b"" if pts[i]["member_start"] else gz.window_of(out, int(pts[i]["out_byte"]))
        assert b"".join(gz.inflate_from(pts, i, w, fetch)) == raw[int(pts[i]["out_byte"]):], i


def test_corrupt_and_truncated():
    blob = gzip.compress(b"abc\n" * 100000)
    with pytest.raises(ValueError):
        gz.build_index(blob[: len(blob) // 2])
    bad = bytearray(blob)
    bad[100:120] = b"\xff" * 20
    with pytest.raises(ValueError):
        gz.build_index(bytes(bad))


def _co_with_index(raw: bytes, blob: bytes, span: int, name: str):
    store = f"gz_{name}"
    MemoryStore._named.pop(store, None)
    co = CloudObject.from_s3(ffq.FASTQGZip, f"s3://b/{name}", fetch=False, s3_config={"endpoint_url": f"memory://{store}"})
    st = co.storage
    st.create_bucket(Bucket="b")
    st.create_bucket(Bucket="b.meta")
    st.put_object(Body=blob, Bucket="b", Key=name)
    inflated, pts = gz.build_index(blob, span=span)
    nl = np.flatnonzero(inflated == 10).astype(np.uint64)
    rows, windows = fgz.window_table(inflated, pts, nl)
    st.put_object(Body=windows, Bucket="b.meta", Key=name + ".idx")
    import pandas as pd
    buf = io.BytesIO()
    pd.DataFrame(rows, columns=fgz.WINDOW_COLUMNS).set_index(["window"]).to_parquet(buf, engine="pyarrow")
    buf.seek(0)
    total = len(nl) + (1 if inflated[-1] != 10 else 0)
    upload_metadata(co, PreprocessingMetadata(metadata=buf, attributes={"total_lines": total,
                                                                        "index_key": name + ".idx"}))
    co.fetch()
    return co


@pytest.mark.parametrize("span,batches", [(1 << 15, 7), (1 << 18, 3), (1 << 22, 5), (1 << 15, 64)])
def test_read_batches_resume(span, batches):
    raw = _raw(20000, 5)
    co = _co_with_index(raw, _multi(raw), span, f"r{span}_{batches}.fq.gz")
    lines = [x.decode() for x in raw.split(b"\n")[:-1]]
    assert co.attributes.total_lines == len(lines)
    sl = co.partition(ffq.partition_reads_batches, num_batches=batches)
    got = []
    for s in sl:
        part = s.get()
        assert len(part) == s.line_1 - s.line_0
        got += part
    assert got == lines


def test_chunk_lines_arbitrary_starts():
    raw = _raw(5000, 9)
    co = _co_with_index(raw, gzip.compress(raw, 6), 1 << 14, "cl.fq.gz")
    lines = [x.decode() for x in raw.split(b"\n")[:-1]]
    for l0 in (1, 2, 3, 777, 4999, 19_997):
        s = fgz.GZipTextSlice(l0, l0 + 5)
        s.cloud_object = co
        assert s.get() == lines[l0 - 1:l0 - 1 + 5]
