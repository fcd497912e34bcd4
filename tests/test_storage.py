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
