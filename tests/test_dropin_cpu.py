"""co.preprocess() plumbing on CPU over the loopback S3 server: storage layout, attrs namedtuple, partial
cleanup, force/skip, and the reference's assertions.  The HIP scan is replaced by a stub serving the
golden index of the sample (fixture data), so this checks host logic only; the GPU tests
(test_gpu_dropin.py) run the same flows through libdpscan."""
import os
import pickle

import numpy as np
import pytest

from dataplug_amd.cloudobject import CloudObject
from dataplug_amd.formats.genomics import fasta as ffa
from dataplug_amd.scan import objects as scan_objects
from dataplug_amd.storage import LoopbackS3Server

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def server():
    with LoopbackS3Server() as srv:
        yield srv


@pytest.fixture(scope="module")
def sample(fasta_cases):
    z = fasta_cases
    i = list(z["kind"]).index("sample")
    data = bytes(z["data"][z["data_off"][i]:z["data_off"][i + 1]])
    exp = z["expected"][z["expected_off"][i]:z["expected_off"][i + 1]].reshape(-1, 2)
    return data, exp


@pytest.fixture
def stub_scan(monkeypatch, sample):
    _, exp = sample
    calls = []

    def in_chunk(c0, c1):
        return exp[(exp[:, 0] >= c0) & (exp[:, 0] < c1)]

    def fasta_index_object(co, plan, u64=False, max_devices=None):
        calls.append(("object", list(plan)))
        return np.concatenate([in_chunk(c0, c1) for c0, c1 in plan])

    def fasta_index_chunk(co, data, chunk_offset, job=0, u64=False):
        calls.append(("chunk", chunk_offset, len(data)))
        return in_chunk(chunk_offset, chunk_offset + len(data))

    monkeypatch.setattr(scan_objects, "fasta_index_object", fasta_index_object)
    monkeypatch.setattr(scan_objects, "fasta_index_chunk", fasta_index_chunk)
    return calls


def _upload(server, data, key="fasta_sample.fasta"):
    co = CloudObject.from_s3(ffa.FASTA, f"s3://genomics/{key}", fetch=False, s3_config=server.storage_config)
    try:
        co.storage.head_bucket(Bucket="genomics")
    except Exception:
        co.storage.create_bucket(Bucket="genomics")
    co.storage.put_object(Body=data, Bucket="genomics", Key=key)
    return CloudObject.from_s3(ffa.FASTA, f"s3://genomics/{key}", s3_config=server.storage_config)


@pytest.mark.parametrize("parallel_config", [{}, {"verbose": 10}, {"backend": "threading", "n_jobs": 4},
                                             {"backend": "sequential"}])
def test_preprocess_layout(server, sample, stub_scan, parallel_config):
    data, exp = sample
    key = f"s{len(parallel_config)}_{parallel_config.get('backend', 'batch')}.fasta"
    co = _upload(server, data, key)
    assert co.exists() and not co.is_preprocessed()
    co.preprocess(parallel_config=parallel_config, chunk_size=-(-len(data) // 4))
    assert co.is_preprocessed()
    st = co.storage
    meta = st.get_object(Bucket="genomics.meta", Key=key)
    assert meta["Metadata"] == {"dataplug": "1.0.0"}
    assert np.array_equal(np.frombuffer(meta["Body"].read(), np.uint32), exp.reshape(-1))
    attrs = pickle.loads(st.get_object(Bucket="genomics.meta", Key=key + ".attrs")["Body"].read())
    assert attrs == {"num_sequences": 9}
    assert type(co.attributes).__name__ == "FASTAAttributes" and co.attributes.num_sequences == 9
    assert co["num_sequences"] == 9 and co.get_attribute("num_sequences") == 9
    left = [c["Key"] for c in st.list_objects_v2(Bucket="genomics.meta")["Contents"] if ".chunk" in c["Key"]]
    assert left == []                                              # partials deleted by the reduce
    kinds = {c[0] for c in stub_scan}
    assert kinds == ({"object"} if "backend" not in parallel_config else {"chunk"})


def test_preprocess_skip_and_force(server, sample, stub_scan):
    data, _ = sample
    co = _upload(server, data, "force.fasta")
    co.preprocess(chunk_size=1000)
    n = len(stub_scan)
    co.preprocess(chunk_size=1000)                 # already preprocessed: no work
    assert len(stub_scan) == n
    co.preprocess(chunk_size=1000, force=True)
    assert len(stub_scan) == n + 1
    assert stub_scan[-1][1] == [(0, 1000), (1000, 2000)]     # num_chunks = size // chunk_size (tail dropped)


def test_preprocess_assertions(server, sample, stub_scan):
    data, _ = sample
    co = _upload(server, data, "asserts.fasta")
    with pytest.raises(AssertionError):
        co.preprocess(chunk_size=0)
    with pytest.raises(AssertionError):
        co.preprocess(chunk_size=len(data) + 1)
    with pytest.raises(KeyError):                  # from_s3 fetches: a missing object is a KeyError
        CloudObject.from_s3(ffa.FASTA, "s3://genomics/missing.fasta", s3_config=server.storage_config)
    missing = CloudObject.from_s3(ffa.FASTA, "s3://genomics/missing.fasta", fetch=False,
                                  s3_config=server.storage_config)
    assert not missing.exists()
    with pytest.raises(AssertionError):
        missing.preprocess(chunk_size=10)


def test_chunk_size_quirk_plan(server, sample, stub_scan):
    # chunk_size == num_chunks - 1  ->  every chunk reads to EOF (handler.py:36-38)
    data, _ = sample
    co = _upload(server, data[:42], "quirk.fasta")       # size 42, cs 6 -> 7 chunks, cs == 7 - 1
    co.preprocess(chunk_size=6)
    assert stub_scan[-1][1] == [(i * 6, 42) for i in range(7)]


def test_partition_after_preprocess(server, sample, stub_scan):
    data, _ = sample
    co = _upload(server, data, "part.fasta")
    co.preprocess(chunk_size=534)
    slices = co.partition(ffa.partition_chunks_strategy, num_chunks=8)
    assert len(slices) == 8 and all(s.cloud_object is co for s in slices)
    assert b"".join(s.get() for s in slices[:1]).startswith(b">")


def test_open_split_header_readline(server, sample):
    data, _ = sample
    co = _upload(server, data, "open.fasta")
    with co.open("rb") as f:
        f.seek(236)
        line = f.readline()
        assert line.startswith(b">") and f.tell() == 296
