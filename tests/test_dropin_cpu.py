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
    for bucket in ("genomics", "genomics.meta"):     # the index bucket too: tests may run alone (-k)
        try:
            co.storage.head_bucket(Bucket=bucket)
        except Exception:
            co.storage.create_bucket(Bucket=bucket)
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


# ------------------------------------------------------------------------------------------ device selection
@pytest.mark.parametrize("where", ["parallel_config", "extra_args"])
def test_device_keyword_ahead_of_env(server, sample, monkeypatch, where):
    """co.preprocess(parallel_config={"dataplug_devices": [...]}) (or the same key in extra_args) picks the
    GPUs ahead of DATAPLUG_AMD_DEVICES, for this call only."""
    data, exp = sample
    seen = []

    def fasta_index_object(co, plan, u64=False, max_devices=None):
        seen.append(scan_objects.devices(max_devices, co))
        return exp

    monkeypatch.setattr(scan_objects, "fasta_index_object", fasta_index_object)
    monkeypatch.setenv("DATAPLUG_AMD_DEVICES", "5,6")
    co = _upload(server, data, f"dev_{where}.fasta")
    kw = {where: {"dataplug_devices": [0, 0, 1]}}
    co.preprocess(chunk_size=534, **kw)
    co.preprocess(chunk_size=534, force=True, **{where: {"dataplug_devices": "2"}})
    co.preprocess(chunk_size=534, force=True, **{where: {"dataplug_devices": 3}})
    co.preprocess(chunk_size=534, force=True)
    assert seen == [[0, 0, 1], [2], [0, 1, 2], [5, 6]]
    assert getattr(co, scan_objects.DEVICES_ATTR) is None
    with pytest.raises(ValueError):
        co.preprocess(chunk_size=534, force=True, **{where: {"dataplug_devices": []}})


def test_device_keyword_reaches_joblib_map_jobs(server, sample, monkeypatch):
    data, exp = sample
    seen = []

    def fasta_index_chunk(co, data, chunk_offset, job=0, u64=False):
        seen.append(tuple(scan_objects.devices(co=co)))
        return exp[(exp[:, 0] >= chunk_offset) & (exp[:, 0] < chunk_offset + len(data))]

    monkeypatch.setattr(scan_objects, "fasta_index_chunk", fasta_index_chunk)
    co = _upload(server, data, "dev_joblib.fasta")
    co.preprocess(chunk_size=534, parallel_config={"backend": "threading", "n_jobs": 2, "dataplug_devices": [1, 0]})
    assert seen and set(seen) == {(1, 0)}
    idx = np.frombuffer(co.storage.get_object(Bucket=co.meta_path.bucket, Key=co.meta_path.key)["Body"].read(),
                        np.uint32)
    assert np.array_equal(idx, exp.reshape(-1))


# ------------------------------------------------------------------------------------------ uint64 index
@pytest.mark.parametrize("parallel_config", [{}, {"backend": "threading", "n_jobs": 2}])
def test_uint64_index_opt_in(server, sample, stub_scan, parallel_config):
    """extra_args={"index_dtype": "uint64"}: same pairs as 8-byte words, attributes say so, and
    partition_chunks_strategy reads it back into the same slices as the uint32 index."""
    data, exp = sample
    co32 = _upload(server, data, "u32.fasta")
    co32.preprocess(chunk_size=534, parallel_config=parallel_config)
    co64 = _upload(server, data, "u64.fasta")
    co64.preprocess(chunk_size=534, parallel_config=parallel_config, extra_args={"index_dtype": "uint64"})
    assert co64.attributes.index_dtype == "uint64" and co64.attributes.num_sequences == 9
    assert not hasattr(co32.attributes, "index_dtype")          # the reference's attributes, unchanged
    raw = co64.storage.get_object(Bucket=co64.meta_path.bucket, Key=co64.meta_path.key)["Body"].read()
    assert np.array_equal(np.frombuffer(raw, "<u8").reshape(-1, 2), exp)
    for n in (1, 3, 8):
        s32 = co32.partition(ffa.partition_chunks_strategy, num_chunks=n)
        s64 = co64.partition(ffa.partition_chunks_strategy, num_chunks=n)
        assert [(s.offset, s.header, s.range_0, s.range_1) for s in s32] == \
            [(s.offset, s.header, s.range_0, s.range_1) for s in s64]
    with pytest.raises(ValueError):
        co64.preprocess(chunk_size=534, force=True, extra_args={"index_dtype": "int8"})


# ------------------------------------------------------------------------------------------ bulk slice gets
def _counting(storage):
    calls = []
    orig = storage.get_object

    def get_object(**kw):
        calls.append(kw.get("Range"))
        return orig(**kw)

    storage.get_object = get_object
    return calls


def test_fasta_get_slices_batched_over_http(server, fasta_cases):
    """get_slices on FASTA slices over the loopback HTTP server: the reference's get() outputs (golden,
    made by running the reference) from a few coalesced ranged GETs instead of 1-2 per slice."""
    import base64
    import json
    from dataplug_amd.entities import get_slices
    from dataplug_amd.preprocessing.handler import upload_metadata
    from dataplug_amd.preprocessing.metadata import PreprocessingMetadata
    from dataplug_amd import synth
    from oracle import cpu_ref
    recs = json.load(open(os.path.join(GOLDEN, "fasta_slices.json")))
    z = fasta_cases
    i = list(z["kind"]).index("sample")
    objs = {"sample": bytes(z["data"][z["data_off"][i]:z["data_off"][i + 1]]),
            "synth1": bytes(synth.fasta(1 << 18, 11))}
    checked = 0
    for rec in recs:
        data = objs[rec["object"]]
        co = _upload(server, data, f"slices_{rec['object']}.fasta")
        idx, nseq = cpu_ref.fasta_index(data, rec["chunk_size"])
        upload_metadata(co, PreprocessingMetadata(metadata=idx, attributes={"num_sequences": nseq}))
        co.fetch()
        slices = co.partition(ffa.partition_chunks_strategy, num_chunks=rec["num_chunks"])
        calls = _counting(co.storage)
        got = get_slices(slices, threads=4)
        n_batched = len(calls)
        if "get" in rec:
            assert [base64.b64encode(g).decode() for g in got] == rec["get"]
        calls.clear()
        assert [s.get() for s in slices] == got
        assert n_batched <= 2 and len(calls) >= len(slices)
        checked += 1
    assert checked == len(recs)


def test_fasta_get_many_in_bounded_groups(server, monkeypatch):
    """FASTASlice.get_many holds one bounded group of coalesced extents at a time: with a tiny
    group size the slices come from several groups and still equal the reference-semantics get()."""
    from dataplug_amd.entities import get_slices
    from dataplug_amd.preprocessing.handler import upload_metadata
    from dataplug_amd.preprocessing.metadata import PreprocessingMetadata
    from dataplug_amd import synth
    from oracle import cpu_ref
    data = bytes(synth.fasta(1 << 18, 11))
    co = _upload(server, data, "slices_grouped.fasta")
    idx, nseq = cpu_ref.fasta_index(data, len(data) // 3 + 1)
    upload_metadata(co, PreprocessingMetadata(metadata=idx, attributes={"num_sequences": nseq}))
    co.fetch()
    slices = co.partition(ffa.partition_chunks_strategy, num_chunks=23)
    monkeypatch.setattr(ffa, "GET_MANY_GROUP_BYTES", 20_000)
    calls = _counting(co.storage)
    got = get_slices(slices, threads=4)
    n_batched = len(calls)
    calls.clear()
    assert got == [s.get() for s in slices]
    assert 5 <= n_batched < len(calls)


def test_force_refreshes_attributes(server, sample, stub_scan):
    """Deliberate deviation: after preprocess(force=True) the in-memory attributes are the
    ones just stored.  The reference's preprocess ends with self.fetch() (cloudobject.py:248), which skips
    _fetch_metadata while _meta_headers is set (:176-178), so a forced re-index of an indexed object keeps
    the previous namedtuple; the stored index and attrs are the same either way."""
    data, exp = sample
    co = _upload(server, data, "force_attrs.fasta")
    co.preprocess(chunk_size=1500)                               # 1 chunk, the tail dropped (num_chunks = size // cs)
    first = co.attributes.num_sequences
    assert first == int(((exp[:, 0] < 1500)).sum()) < 9
    co.preprocess(chunk_size=-(-len(data) // 4), force=True)     # every byte: all 9 headers
    stored = pickle.loads(co.storage.get_object(Bucket="genomics.meta", Key="force_attrs.fasta.attrs")["Body"].read())
    assert stored == {"num_sequences": 9}
    assert co.attributes.num_sequences == 9                      # the reference would still report `first`


def test_get_slices_first_error_in_slice_order():
    from dataplug_amd.entities import CloudObjectSlice, get_slices

    class S(CloudObjectSlice):
        def __init__(self, i):
            super().__init__(i, i + 1)
            self.i = i

        def get(self):
            if self.i in (3, 7):
                raise ValueError(f"slice {self.i}")
            return self.i

    assert get_slices([S(i) for i in (0, 1, 2)], threads=4) == [0, 1, 2]
    with pytest.raises(ValueError, match="slice 3"):
        get_slices([S(i) for i in range(10)], threads=4)


def test_fasta_passes_cover_group_in_order():
    """scan.objects.fasta_passes: consecutive runs of whole chunks within the byte budget (a larger chunk
    alone), covering the group's chunks exactly once, in order, each pass's fetched bytes within budget."""
    from dataplug_amd.scan.objects import FastaGroup, fasta_passes
    size = 10_000_000
    plan = [(i * 700_000, min(size, (i + 1) * 700_000)) for i in range(15)]
    g = FastaGroup(2, 13, plan[2][0], plan[12][1], min(size, plan[12][1] + 65_536))
    for budget in (1 << 40, 3_000_000, 800_000, 100):
        ps = fasta_passes(plan, g, size, budget)
        assert ps[0].i0 == g.i0 and ps[-1].i1 == g.i1
        assert all(a.i1 == b.i0 for a, b in zip(ps, ps[1:]))
        for p in ps:
            assert p.lo == min(c0 for c0, _ in plan[p.i0:p.i1]) and p.hi == max(c1 for _, c1 in plan[p.i0:p.i1])
            assert p.buf_hi - p.lo <= budget or p.i1 - p.i0 == 1
        if budget == 1 << 40:
            assert ps == [g]
    # the reference's cs == n - 1 quirk: every chunk reads to EOF, so every chunk is a pass of its own
    quirk = [(i * 3, size) for i in range(4)]
    gq = FastaGroup(0, 4, 0, size, size)
    assert [(p.i0, p.i1) for p in fasta_passes(quirk, gq, size, size // 2)] == [(0, 1), (1, 2), (2, 3), (3, 4)]
