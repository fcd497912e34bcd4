"""Storage surface of the indexing path: in-process and loopback-HTTP S3 behave alike."""
import copy
import io
import pickle

import pytest

from dataplug_amd.storage import (ClientError, LoopbackS3Server, MemoryStore, PickleableS3ClientProxy, S3Path,
                                  make_client, open_object, parse_range)


@pytest.fixture(scope="module")
def server():
    with LoopbackS3Server() as srv:
        yield srv


@pytest.fixture(params=["memory", "http"])
def client(request, server):
    if request.param == "memory":
        name = f"t{id(request)}"
        MemoryStore._named.pop(name, None)
        return make_client(f"memory://{name}")
    return make_client(server.endpoint_url)


def test_s3path():
    p = S3Path.from_uri("s3://genomics/dir/a/../fasta_sample.fasta")
    assert (p.bucket, p.key) == ("genomics", "dir/fasta_sample.fasta")
    assert p.as_uri() == "s3://genomics/dir/fasta_sample.fasta"
    assert p.virtual_directory == "dir"
    assert S3Path.from_bucket_key("b.meta", "k.attrs").as_uri() == "s3://b.meta/k.attrs"
    assert pickle.loads(pickle.dumps(p)) == p
    with pytest.raises(ValueError):
        S3Path.from_uri("http://x/y")


@pytest.mark.parametrize("rng,size,exp", [
    (None, 10, None), ("bytes=0-0", 10, (0, 1)), ("bytes=2-5", 10, (2, 6)), ("bytes=8-100", 10, (8, 10)),
    ("bytes=3-", 10, (3, 10)), ("bytes=-4", 10, (6, 10)),
])
def test_parse_range(rng, size, exp):
    assert parse_range(rng, size) == exp


def test_parse_range_unsatisfiable():
    with pytest.raises(ClientError) as e:
        parse_range("bytes=10-12", 10)
    assert e.value.response["Error"]["Code"] == "InvalidRange"


def test_bucket_and_object_roundtrip(client):
    with pytest.raises(ClientError) as e:
        client.head_bucket(Bucket="b")
    assert e.value.response["Error"]["Code"] == "404"
    client.create_bucket(Bucket="b")
    assert client.head_bucket(Bucket="b")["ResponseMetadata"]["HTTPStatusCode"] == 200
    data = bytes(range(256)) * 1000
    client.put_object(Body=data, Bucket="b", Key="dir/obj", Metadata={"dataplug": "1.0.0"})
    h = client.head_object(Bucket="b", Key="dir/obj")
    assert h["ContentLength"] == len(data) and h["Metadata"] == {"dataplug": "1.0.0"}
    r = client.get_object(Bucket="b", Key="dir/obj")
    assert r["ResponseMetadata"]["HTTPStatusCode"] == 200 and r["Body"].read() == data
    r = client.get_object(Bucket="b", Key="dir/obj", Range="bytes=1000-1999")   # inclusive
    assert r["ResponseMetadata"]["HTTPStatusCode"] == 206 and r["Body"].read() == data[1000:2000]
    r = client.get_object(Bucket="b", Key="dir/obj", Range=f"bytes={len(data) - 5}-{len(data) + 100}")
    assert r["Body"].read() == data[-5:]
    body = client.get_object(Bucket="b", Key="dir/obj", Range="bytes=0-99999")["Body"]
    buf = bytearray(100000)
    got = 0
    while got < len(buf):
        got += body.readinto(memoryview(buf)[got:])
    assert bytes(buf) == data[:100000]
    with pytest.raises(ClientError) as e:
        client.head_object(Bucket="b", Key="missing")
    assert e.value.response["Error"]["Code"] == "404"
    with pytest.raises(ClientError) as e:
        client.get_object(Bucket="b", Key="missing")
    assert e.value.response["Error"]["Code"] == "NoSuchKey"
    client.upload_fileobj(io.BytesIO(b"abc"), "b", "up", ExtraArgs={"Metadata": {"k": "v"}})
    assert client.head_object(Bucket="b", Key="up")["Metadata"] == {"k": "v"}
    keys = [c["Key"] for c in client.list_objects_v2(Bucket="b")["Contents"]]
    assert keys == ["dir/obj", "up"]
    client.delete_object(Bucket="b", Key="up")
    assert [c["Key"] for c in client.list_objects_v2(Bucket="b")["Contents"]] == ["dir/obj"]


def test_open_object_seek_readline(client):
    client.create_bucket(Bucket="b")
    data = b">h1 x\nACGT\n>h2\nGG\n"
    client.put_object(Body=data, Bucket="b", Key="f")
    with open_object(client, "b", "f", "rb", buffer_size=4) as f:
        f.seek(11)
        assert f.readline() == b">h2\n" and f.tell() == 15
        f.seek(0)
        assert f.read() == data
    with open_object(client, "b", "f", "r") as f:
        assert f.readline() == ">h1 x\n"


def test_proxy_pickle_and_deepcopy(server):
    p = PickleableS3ClientProxy(endpoint_url=server.endpoint_url, role_arn="arn:aws:iam::1:role/x")
    p.create_bucket(Bucket="px")
    p.put_object(Body=b"1", Bucket="px", Key="k")
    q = pickle.loads(pickle.dumps(p))
    assert q.get_object(Bucket="px", Key="k")["Body"].read() == b"1"
    r = copy.deepcopy(p)
    assert r.head_object(Bucket="px", Key="k")["ContentLength"] == 1
    m = PickleableS3ClientProxy(endpoint_url="memory://proxy_test")
    m.create_bucket(Bucket="m")
    m.put_object(Body=b"zz", Bucket="m", Key="k")
    assert copy.deepcopy(m).get_object(Bucket="m", Key="k")["Body"].read() == b"zz"


def test_proxy_requires_endpoint(monkeypatch):
    monkeypatch.delenv("DATAPLUG_S3_ENDPOINT", raising=False)
    with pytest.raises(ValueError):
        PickleableS3ClientProxy()


def test_put_buffer_bodies(client):
    """Array bodies go up without a copy on the client side (a flat byte view) and read back as their bytes;
    the stored object does not follow later writes to the caller's array."""
    import numpy as np
    client.create_bucket(Bucket="arr")
    a = np.arange(1000, dtype="<u8")
    client.put_object(Body=a.data, Bucket="arr", Key="c")
    client.put_object(Body=a[::3], Bucket="arr", Key="s")              # non-contiguous: copied
    client.put_object(Body=np.zeros(0, np.uint8), Bucket="arr", Key="e")
    want = a.tobytes()
    a[:] = 7
    assert client.get_object(Bucket="arr", Key="c")["Body"].read() == want
    assert client.get_object(Bucket="arr", Key="s")["Body"].read() == np.arange(1000, dtype="<u8")[::3].tobytes()
    assert client.get_object(Bucket="arr", Key="e")["Body"].read() == b""
    assert client.head_object(Bucket="arr", Key="c")["ContentLength"] == 8000


def test_memory_store_owned_put():
    st = MemoryStore()
    st.create_bucket("b")
    src = bytearray(b"abc")
    assert st.put("b", "copied", src).data == b"abc"
    src[0] = ord("x")
    assert st.get("b", "copied").data == b"abc"                          # a copy unless handed over
    kept = bytearray(b"def")
    assert st.put("b", "owned", kept, owned=True).data is kept


def test_store_line_index_u8s(client):
    """The u8s index's three objects (low bytes here, counts and block table on the side thread) and its
    attributes; a failed PUT (no such bucket) raises from the call."""
    import numpy as np
    from dataplug_amd.formats._lines import store_line_index
    from dataplug_amd.scan.objects import ByteOffsets
    from dataplug_amd.storage import S3Path

    class Co:
        storage = client
        meta_path = S3Path.from_bucket_key("idx.meta", "obj")
    client.create_bucket(Bucket="idx.meta")
    off = ByteOffsets(np.arange(5, dtype=np.uint8), np.asarray([0, 5], np.uint16), np.asarray([0], np.uint64), 0, 0)
    attrs = store_line_index(Co, off)
    assert attrs["line_index_dtype"] == "u8s" and attrs["num_lines"] == 5

    def get(key):
        return client.get_object(Bucket="idx.meta", Key=key)["Body"].read()
    assert get(attrs["line_index_key"]) == bytes(range(5))
    assert get(attrs["line_index_sub_key"]) == np.asarray([0, 5], "<u2").tobytes()
    assert get(attrs["line_index_blocks_key"]) == np.zeros(1, "<u8").tobytes()

    class Missing(Co):
        meta_path = S3Path.from_bucket_key("no-such-bucket.meta", "obj")
    with pytest.raises(ClientError):
        store_line_index(Missing, off)


def test_multipart_upload(client):
    """S3 multipart uploads (the streamed index PUT): parts in order, every one but the last >= 5 MiB; ranged reads
    inside one part and across part boundaries; metadata from the create call; an aborted upload is gone; a part
    below the minimum is refused at completion."""
    import numpy as np
    client.create_bucket(Bucket="mp")
    rng = np.random.default_rng(2)
    parts = [rng.integers(0, 256, n, dtype=np.uint8) for n in (5 << 20, (6 << 20) + 3, 1234)]
    uid = client.create_multipart_upload(Bucket="mp", Key="o", Metadata={"dataplug": "1.0.0"})["UploadId"]
    etags = [client.upload_part(Bucket="mp", Key="o", PartNumber=i + 1, UploadId=uid, Body=p.data)["ETag"]
             for i, p in enumerate(parts)]
    client.complete_multipart_upload(Bucket="mp", Key="o", UploadId=uid, MultipartUpload={
        "Parts": [{"PartNumber": i + 1, "ETag": e} for i, e in enumerate(etags)]})
    whole = np.concatenate(parts).tobytes()
    h = client.head_object(Bucket="mp", Key="o")
    assert h["ContentLength"] == len(whole) and h["Metadata"] == {"dataplug": "1.0.0"}
    assert client.get_object(Bucket="mp", Key="o")["Body"].read() == whole
    for a, b in [(0, 9), ((5 << 20) - 3, (5 << 20) + 6), (100, (11 << 20) + 200), (len(whole) - 5, len(whole) - 1)]:
        assert client.get_object(Bucket="mp", Key="o", Range=f"bytes={a}-{b}")["Body"].read() == whole[a:b + 1]
    uid = client.create_multipart_upload(Bucket="mp", Key="gone")["UploadId"]
    client.upload_part(Bucket="mp", Key="gone", PartNumber=1, UploadId=uid, Body=b"x" * 10)
    client.abort_multipart_upload(Bucket="mp", Key="gone", UploadId=uid)
    with pytest.raises(ClientError) as ei:
        client.upload_part(Bucket="mp", Key="gone", PartNumber=2, UploadId=uid, Body=b"y")
    assert ei.value.response["Error"]["Code"] == "NoSuchUpload"
    with pytest.raises(ClientError):
        client.head_object(Bucket="mp", Key="gone")
    uid = client.create_multipart_upload(Bucket="mp", Key="small")["UploadId"]
    for i in (1, 2):
        client.upload_part(Bucket="mp", Key="small", PartNumber=i, UploadId=uid, Body=b"z" * 100)
    with pytest.raises(ClientError) as ei:
        client.complete_multipart_upload(Bucket="mp", Key="small", UploadId=uid, MultipartUpload={
            "Parts": [{"PartNumber": 1, "ETag": ""}, {"PartNumber": 2, "ETag": ""}]})
    assert ei.value.response["Error"]["Code"] == "EntityTooSmall"


@pytest.mark.parametrize("fmt", ["u8s", "u16b"])
def test_streamed_index_equals_stored_index(client, monkeypatch, fmt):
    """verdict r5 #4: the index stored piece by piece while later pieces are scanned (multipart low bytes and
    256-byte counts, the block table at the end) is byte-identical to the merged index stored at once, and
    LineIndex reads every offset back.  Each piece's GPU scan replaced by what the kernel returns for it (host logic
    only: the piece split over the device entries' workers, the ordered merge and the uploads)."""
    import numpy as np
    from types import SimpleNamespace
    from test_partition_golden import byte_offsets
    from dataplug_amd.formats import _lines
    from dataplug_amd.scan import objects
    G = 1 << 30
    rng = np.random.default_rng(8)
    begin, end = G + 4321, 3 * G + 77
    off = np.unique(rng.integers(begin, end, 6_500_000).astype(np.uint64))

    def fake_group(dev, co, lo, hi, delim, every_k, emit_add, fmt="u64"):
        sel = off[(off >= lo) & (off < hi)]
        if fmt == "u8s":
            bo = byte_offsets(sel, lo, hi)
            return bo.low, bo.table, bo.sub
        j0 = lo >> 16
        tab = np.searchsorted(sel, (np.arange(j0, ((hi - 1) >> 16) + 1, dtype=np.uint64) << np.uint64(16))).astype(np.uint64)
        if lo & 0xFFFF:
            tab[0] = 0
        return (sel & np.uint64(0xFFFF)).astype(np.uint16), tab
    def fake_run(dev, co, jobs, delim, fmt_, stop):
        for lo, hi, fut in jobs:                       # in order, as the device worker runs them
            fut.set_result(fake_group(dev, co, lo, hi, delim, 1, 0, fmt=fmt_))
    monkeypatch.setattr(objects, "_delim_group", fake_group)
    monkeypatch.setattr(objects, "_delim_piece_run", fake_run)
    monkeypatch.setattr(_lines, "PART_MIN", 5 << 20)
    monkeypatch.setenv("DATAPLUG_AMD_DEVICES", "0,0")
    client.create_bucket(Bucket="ds")
    client.create_bucket(Bucket="ds.meta")

    def co_for(key):
        return SimpleNamespace(size=end, storage=client, path=SimpleNamespace(bucket="ds", key=key),
                               meta_path=SimpleNamespace(bucket="ds.meta", key=key))
    a = _lines.index_object(co_for("streamed"), begin, fmt, piece_bytes=(G // 3) + 11)
    b = _lines.store_line_index(co_for("whole"), objects.line_index_object(co_for("whole"), begin, end, fmt=fmt,
                                                                           part_bytes=(G // 2) + 5))
    assert a["num_lines"] == b["num_lines"] == len(off) and a["line_index_dtype"] == b["line_index_dtype"] == fmt
    for attr in ("line_index_key", "line_index_blocks_key") + (("line_index_sub_key",) if fmt == "u8s" else ()):
        got = client.get_object(Bucket="ds.meta", Key=a[attr])["Body"].read()
        assert got == client.get_object(Bucket="ds.meta", Key=b[attr])["Body"].read(), attr
    assert {k: v for k, v in a.items() if not k.endswith("_key")} == {k: v for k, v in b.items() if not k.endswith("_key")}
    blocks = np.frombuffer(client.get_object(Bucket="ds.meta", Key=a["line_index_blocks_key"])["Body"].read(), "<u8")
    li = _lines.LineIndex(storage=client, bucket="ds.meta", key=a["line_index_key"], count=a["num_lines"], blocks=blocks,
                          block0=a["line_index_block0"], sub_key=a.get("line_index_sub_key"), sub0=a.get("line_index_sub0", 0))
    assert np.array_equal(li._fetch(0, li.count), off)
