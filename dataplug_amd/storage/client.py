"""boto3-shaped S3 clients without boto3: in-process (``memory://name``) and HTTP (S3 REST, path style).

The indexing path uses this storage surface: ``head_object`` (404 → ``ClientError``
code ``"404"``), ``head_bucket``, ``create_bucket``, ``get_object(Range="bytes=a-b")`` (inclusive; body
with ``.read()``; status 200/206), ``put_object``, ``upload_fileobj``, ``upload_file``, ``download_file``,
``delete_object``, and the multipart upload calls (``create_multipart_upload``, ``upload_part``,
``complete_multipart_upload``, ``abort_multipart_upload``) the streamed index PUT uses.  ``PickleableS3ClientProxy`` takes the reference's ``storage_config`` keywords
(``picklableS3.py:49-84``) and re-creates its client after pickling, like the reference's proxy.

Scope: unsigned requests to S3-compatible endpoints (the loopback server in ``server.py``, MinIO with
anonymous access).  AWS SigV4 / STS role assumption is the reference's auth layer and out of scope.
"""
from __future__ import annotations

import http.client
import io
import os
import shutil
import threading
import urllib.parse
import xml.etree.ElementTree as ET
from email.utils import formatdate
from typing import Dict, Optional

import numpy as np

from .errors import ClientError
from .memory import MemoryStore, parse_range

_COPY_BLOCK = 8 << 20


class StreamingBody(io.RawIOBase):
    """File-like response body: ``read([n])``, ``readinto(buf)``, ``close()``."""

    def __init__(self, src, length: int, on_close=None):
        self._src = src                  # memoryview (in-process) or HTTPResponse
        self._len = int(length)
        self._pos = 0
        self._on_close = on_close

    @property
    def content_length(self) -> int:
        return self._len

    def readable(self) -> bool:
        return True

    def readinto(self, b) -> int:
        n = min(len(b), self._len - self._pos)
        if n <= 0:
            return 0
        if isinstance(self._src, memoryview):
            # numpy copies without holding the GIL, so parallel ranged GETs copy in parallel
            np.copyto(np.frombuffer(memoryview(b).cast("B")[:n], np.uint8),
                      np.frombuffer(self._src[self._pos:self._pos + n], np.uint8))
        else:
            n = self._src.readinto(memoryview(b).cast("B")[:n])
            if n == 0:
                raise IOError(f"connection closed after {self._pos} of {self._len} bytes")
        self._pos += n
        return n

    def read(self, amt: Optional[int] = None) -> bytes:
        left = self._len - self._pos
        n = left if amt is None or amt < 0 else min(amt, left)
        if n <= 0:
            return b""
        if isinstance(self._src, memoryview):
            out = bytes(self._src[self._pos:self._pos + n])
            self._pos += n
            return out
        buf = bytearray(n)
        view = memoryview(buf)
        got = 0
        while got < n:
            got += self.readinto(view[got:])
        return bytes(buf)

    def readall(self) -> bytes:
        return self.read()

    def close(self) -> None:
        if not self.closed:
            if self._on_close is not None:
                self._on_close()
            super().close()


def _meta_from(extra_args: Optional[dict]) -> Dict[str, str]:
    return dict((extra_args or {}).get("Metadata") or {})


def _body_bytes(body):
    """A PUT body as bytes, or as a flat byte view of a contiguous buffer (no copy: an HTTP request sends it as it
    is, the memory store copies it into its own bytes)."""
    if body is None:
        return b""
    if isinstance(body, str):
        return body.encode("utf-8")
    if hasattr(body, "read"):
        return body.read()
    if isinstance(body, bytes):
        return body
    try:
        return memoryview(body).cast("B")
    except TypeError:                             # (a non-contiguous buffer)
        return bytes(body)


class _ClientBase:
    """boto3 method names and shapes on top of five primitives implemented by the subclasses."""

    # primitives: _head(b, k) -> (size, meta, etag, mtime); _get(b, k, rng) -> (body, size, total, meta, status);
    # _put(b, k, data|file, size, meta); _delete(b, k); _head_bucket(b) -> bool; _create_bucket(b); _list(b, prefix);
    # multipart: _mp_create(b, k, meta) -> id; _mp_part(b, k, id, n, data, size) -> etag; _mp_complete(b, k, id, [n]);
    # _mp_abort(b, k, id)

    def head_bucket(self, Bucket: str, **_):
        if not self._head_bucket(Bucket):
            raise ClientError("404", "HeadBucket", Bucket)
        return {"ResponseMetadata": {"HTTPStatusCode": 200}}

    def create_bucket(self, Bucket: str, **_):
        self._create_bucket(Bucket)
        return {"Location": f"/{Bucket}", "ResponseMetadata": {"HTTPStatusCode": 200}}

    def head_object(self, Bucket: str, Key: str, **_):
        size, meta, etag, mtime = self._head(Bucket, Key)
        return {"ContentLength": size, "ETag": etag, "LastModified": mtime, "Metadata": meta,
                "ContentType": "binary/octet-stream", "ResponseMetadata": {"HTTPStatusCode": 200}}

    def get_object(self, Bucket: str, Key: str, Range: Optional[str] = None, **_):
        body, n, total, meta, status, lo = self._get(Bucket, Key, Range)
        res = {"Body": body, "ContentLength": n, "Metadata": meta,
               "ResponseMetadata": {"HTTPStatusCode": status}}
        if status == 206:
            res["ContentRange"] = f"bytes {lo}-{lo + n - 1}/{total}"
        return res

    def put_object(self, Bucket: str, Key: str, Body=None, Metadata: Optional[Dict[str, str]] = None, **_):
        data = _body_bytes(Body)
        self._put(Bucket, Key, data, len(data), dict(Metadata or {}))
        return {"ResponseMetadata": {"HTTPStatusCode": 200}}

    def create_multipart_upload(self, Bucket: str, Key: str, Metadata: Optional[Dict[str, str]] = None, **_):
        uid = self._mp_create(Bucket, Key, dict(Metadata or {}))
        return {"Bucket": Bucket, "Key": Key, "UploadId": uid, "ResponseMetadata": {"HTTPStatusCode": 200}}

    def upload_part(self, Bucket: str, Key: str, PartNumber: int, UploadId: str, Body=None, **_):
        data = _body_bytes(Body)
        etag = self._mp_part(Bucket, Key, UploadId, int(PartNumber), data, len(data))
        return {"ETag": etag, "ResponseMetadata": {"HTTPStatusCode": 200}}

    def complete_multipart_upload(self, Bucket: str, Key: str, UploadId: str, MultipartUpload: dict, **_):
        numbers = [int(p["PartNumber"]) for p in MultipartUpload.get("Parts", [])]
        self._mp_complete(Bucket, Key, UploadId, numbers)
        return {"Bucket": Bucket, "Key": Key, "ResponseMetadata": {"HTTPStatusCode": 200}}

    def abort_multipart_upload(self, Bucket: str, Key: str, UploadId: str, **_):
        self._mp_abort(Bucket, Key, UploadId)
        return {"ResponseMetadata": {"HTTPStatusCode": 204}}

    def delete_object(self, Bucket: str, Key: str, **_):
        self._delete(Bucket, Key)
        return {"ResponseMetadata": {"HTTPStatusCode": 204}}

    def delete_objects(self, Bucket: str, Delete: dict, **_):
        keys = [o["Key"] for o in Delete.get("Objects", [])]
        for k in keys:
            self._delete(Bucket, k)
        return {"Deleted": [{"Key": k} for k in keys], "ResponseMetadata": {"HTTPStatusCode": 200}}

    def list_objects_v2(self, Bucket: str, Prefix: str = "", **_):
        items = [{"Key": k, "Size": s} for k, s in self._list(Bucket, Prefix)]
        return {"Contents": items, "KeyCount": len(items), "IsTruncated": False,
                "ResponseMetadata": {"HTTPStatusCode": 200}}

    list_objects = list_objects_v2

    def upload_fileobj(self, Fileobj, Bucket: str, Key: str, ExtraArgs: Optional[dict] = None, Callback=None,
                       Config=None):
        data = Fileobj.read()
        if isinstance(data, str):
            data = data.encode("utf-8")
        self._put(Bucket, Key, data, len(data), _meta_from(ExtraArgs))
        if Callback is not None:
            Callback(len(data))

    def upload_file(self, Filename: str, Bucket: str, Key: str, ExtraArgs: Optional[dict] = None, Callback=None,
                    Config=None):
        with open(Filename, "rb") as f:
            self.upload_fileobj(f, Bucket, Key, ExtraArgs=ExtraArgs, Callback=Callback)

    def download_fileobj(self, Bucket: str, Key: str, Fileobj, ExtraArgs=None, Callback=None, Config=None):
        body = self.get_object(Bucket=Bucket, Key=Key)["Body"]
        with body:
            shutil.copyfileobj(body, Fileobj, _COPY_BLOCK)

    def download_file(self, Bucket: str, Key: str, Filename: str, ExtraArgs=None, Callback=None, Config=None):
        with open(Filename, "wb") as f:
            self.download_fileobj(Bucket, Key, f)


class LocalS3Client(_ClientBase):
    """In-process client over a ``MemoryStore`` (zero-copy ranged reads)."""

    def __init__(self, store: MemoryStore):
        self.store = store

    def _head_bucket(self, b):
        return self.store.has_bucket(b)

    def _create_bucket(self, b):
        self.store.create_bucket(b)

    def _head(self, b, k):
        try:
            o = self.store.get(b, k, "HeadObject")
        except ClientError as e:
            raise ClientError("404", "HeadObject", str(e)) from None
        return len(o.data), dict(o.metadata), o.etag, o.last_modified

    def _get(self, b, k, rng):
        o = self.store.get(b, k)
        r = parse_range(rng, len(o.data))
        lo, hi = r if r is not None else (0, len(o.data))
        return (StreamingBody(o.view(lo, hi), hi - lo), hi - lo, len(o.data), dict(o.metadata),
                206 if r is not None else 200, lo)

    def _put(self, b, k, data, size, meta):
        self.store.put(b, k, data, meta)

    def _mp_create(self, b, k, meta):
        return self.store.create_multipart(b, k, meta)

    def _mp_part(self, b, k, uid, n, data, size):
        return self.store.upload_part(b, k, uid, n, data)

    def _mp_complete(self, b, k, uid, numbers):
        self.store.complete_multipart(b, k, uid, numbers)

    def _mp_abort(self, b, k, uid):
        self.store.abort_multipart(b, k, uid)

    def _delete(self, b, k):
        self.store.delete(b, k)

    def _list(self, b, prefix):
        return [(k, len(o.data)) for k, o in self.store.list(b, prefix)]


class HTTPS3Client(_ClientBase):
    """Path-style S3 REST over ``http.client`` (one connection per request thread)."""

    def __init__(self, endpoint_url: str, timeout: float = 300.0):
        u = urllib.parse.urlsplit(endpoint_url)
        if u.scheme not in ("http", "https"):
            raise ValueError(f"unsupported endpoint {endpoint_url!r}")
        self.endpoint_url = endpoint_url
        self._https = u.scheme == "https"
        self._host = u.hostname
        self._port = u.port or (443 if self._https else 80)
        self._timeout = timeout
        self._tls = threading.local()

    def _new_conn(self):
        cls = http.client.HTTPSConnection if self._https else http.client.HTTPConnection
        return cls(self._host, self._port, timeout=self._timeout)

    @staticmethod
    def _path(b: str, k: Optional[str] = None, query: str = "") -> str:
        p = "/" + urllib.parse.quote(b, safe="")
        if k is not None:
            p += "/" + urllib.parse.quote(k, safe="/~")
        return p + (("?" + query) if query else "")

    def _request(self, method: str, path: str, body=None, headers=None, op: str = "", stream: bool = False):
        """(response, conn).  Non-streaming responses are fully read; their connection is reused."""
        conn = getattr(self._tls, "conn", None) if not stream else None
        if conn is None:
            conn = self._new_conn()
        hdrs = {"Date": formatdate(usegmt=True)}
        hdrs.update(headers or {})
        try:
            conn.request(method, path, body=body, headers=hdrs)
            resp = conn.getresponse()
        except (http.client.HTTPException, ConnectionError, OSError):
            conn.close()
            if stream or getattr(self._tls, "conn", None) is None:
                raise
            conn = self._new_conn()                       # stale keep-alive connection: retry once
            conn.request(method, path, body=body, headers=hdrs)
            resp = conn.getresponse()
        if resp.status >= 300:
            payload = resp.read()
            conn.close()
            self._tls.conn = None
            code = str(resp.status)
            msg = resp.reason
            if payload:
                try:
                    root = ET.fromstring(payload)
                    code = root.findtext("Code") or code
                    msg = root.findtext("Message") or msg
                except ET.ParseError:
                    pass
            if method == "HEAD" and resp.status == 404:
                code = "404"
            raise ClientError(code, op, msg, resp.status)
        if not stream:
            resp.read()  # drained below by callers that need the payload (they pass stream=True)
            self._tls.conn = conn
        return resp, conn

    def _head_bucket(self, b):
        try:
            self._request("HEAD", self._path(b), op="HeadBucket")
            return True
        except ClientError as e:
            if e.response["ResponseMetadata"]["HTTPStatusCode"] == 404:
                return False
            raise

    def _create_bucket(self, b):
        self._request("PUT", self._path(b), body=b"", headers={"Content-Length": "0"}, op="CreateBucket")

    def _head(self, b, k):
        resp, _ = self._request("HEAD", self._path(b, k), op="HeadObject")
        meta = {h[len("x-amz-meta-"):]: v for h, v in resp.getheaders() if h.lower().startswith("x-amz-meta-")}
        return int(resp.getheader("Content-Length", "0")), meta, resp.getheader("ETag", ""), \
            resp.getheader("Last-Modified", "")

    def _get(self, b, k, rng):
        headers = {"Range": rng} if rng else {}
        resp, conn = self._request("GET", self._path(b, k), headers=headers, op="GetObject", stream=True)
        n = int(resp.getheader("Content-Length", "0"))
        total, lo = n, 0
        cr = resp.getheader("Content-Range")
        if cr:
            span, _, tot = cr.split(" ", 1)[1].partition("/")
            lo = int(span.split("-")[0])
            total = int(tot) if tot != "*" else n
        meta = {h[len("x-amz-meta-"):]: v for h, v in resp.getheaders() if h.lower().startswith("x-amz-meta-")}
        return StreamingBody(resp, n, on_close=conn.close), n, total, meta, resp.status, lo

    def _put(self, b, k, data, size, meta):
        headers = {"Content-Length": str(size), "Content-Type": "binary/octet-stream"}
        headers.update({f"x-amz-meta-{m}": str(v) for m, v in meta.items()})
        self._request("PUT", self._path(b, k), body=data, headers=headers, op="PutObject")

    def _delete(self, b, k):
        self._request("DELETE", self._path(b, k), op="DeleteObject")

    def _mp_create(self, b, k, meta):
        headers = {"Content-Length": "0"}
        headers.update({f"x-amz-meta-{m}": str(v) for m, v in meta.items()})
        resp, conn = self._request("POST", self._path(b, k, "uploads"), body=b"", headers=headers,
                                   op="CreateMultipartUpload", stream=True)
        payload = resp.read()
        self._tls.conn = conn
        root = ET.fromstring(payload)
        uid = next((e.text for e in root.iter() if e.tag.endswith("UploadId")), None)
        if not uid:
            raise ClientError("InternalError", "CreateMultipartUpload", "no UploadId in the response", 500)
        return uid

    def _mp_part(self, b, k, uid, n, data, size):
        q = urllib.parse.urlencode({"partNumber": str(n), "uploadId": uid})
        resp, _ = self._request("PUT", self._path(b, k, q), body=data,
                                headers={"Content-Length": str(size), "Content-Type": "binary/octet-stream"},
                                op="UploadPart")
        return resp.getheader("ETag", "")

    def _mp_complete(self, b, k, uid, numbers):
        body = ("<CompleteMultipartUpload>" + "".join(f"<Part><PartNumber>{n}</PartNumber></Part>" for n in numbers)
                + "</CompleteMultipartUpload>").encode()
        q = urllib.parse.urlencode({"uploadId": uid})
        resp, conn = self._request("POST", self._path(b, k, q), body=body,
                                   headers={"Content-Length": str(len(body)), "Content-Type": "application/xml"},
                                   op="CompleteMultipartUpload", stream=True)
        payload = resp.read()
        self._tls.conn = conn
        if b"<Error>" in payload:                 # S3 may answer 200 with an error document
            root = ET.fromstring(payload)
            raise ClientError(root.findtext("Code") or "InternalError", "CompleteMultipartUpload",
                              root.findtext("Message") or "", 500)

    def _mp_abort(self, b, k, uid):
        self._request("DELETE", self._path(b, k, urllib.parse.urlencode({"uploadId": uid})),
                      op="AbortMultipartUpload")

    def _list(self, b, prefix):
        q = urllib.parse.urlencode({"list-type": "2", "prefix": prefix})
        resp, conn = self._request("GET", self._path(b, query=q), op="ListObjectsV2", stream=True)
        payload = resp.read()
        conn.close()
        root = ET.fromstring(payload)
        out = []
        for c in root.iter():
            if c.tag.endswith("Contents"):
                key = size = None
                for e in c:
                    if e.tag.endswith("Key"):
                        key = e.text
                    elif e.tag.endswith("Size"):
                        size = int(e.text)
                out.append((key, size))
        return out

    def upload_fileobj(self, Fileobj, Bucket: str, Key: str, ExtraArgs: Optional[dict] = None, Callback=None,
                       Config=None):
        # stream seekable files without loading them (http.client sends file bodies in blocks)
        if hasattr(Fileobj, "seek") and hasattr(Fileobj, "tell") and not isinstance(Fileobj, io.TextIOBase):
            pos = Fileobj.tell()
            Fileobj.seek(0, io.SEEK_END)
            size = Fileobj.tell() - pos
            Fileobj.seek(pos)
            self._put(Bucket, Key, Fileobj, size, _meta_from(ExtraArgs))
            if Callback is not None:
                Callback(size)
            return
        super().upload_fileobj(Fileobj, Bucket, Key, ExtraArgs=ExtraArgs, Callback=Callback)


def make_client(endpoint_url: Optional[str]):
    if endpoint_url is None:
        endpoint_url = os.environ.get("DATAPLUG_S3_ENDPOINT")
    if not endpoint_url:
        raise ValueError("storage_config needs an 'endpoint_url' (http://host:port of an S3-compatible endpoint, "
                         "or memory://<name> for an in-process store); AWS SigV4/STS is out of scope")
    if endpoint_url.startswith("memory://"):
        return LocalS3Client(MemoryStore.named(endpoint_url[len("memory://"):] or "default"))
    return HTTPS3Client(endpoint_url)


class PickleableS3ClientProxy:
    """The reference's client proxy contract (picklableS3.py:36-190): construct from ``storage_config``
    keywords, expose the boto3 client methods, survive pickling/deepcopy by re-creating the client."""

    def __init__(self, region_name: Optional[str] = None, endpoint_url: Optional[str] = None,
                 credentials: Optional[dict] = None, role_arn: Optional[str] = None,
                 token_duration_seconds: Optional[int] = None, botocore_config_kwargs: Optional[dict] = None,
                 client=None):
        self.region_name = region_name
        self.endpoint_url = endpoint_url if endpoint_url is not None else os.environ.get("DATAPLUG_S3_ENDPOINT")
        self.credentials = credentials
        self.role_arn = role_arn
        self.token_duration_seconds = token_duration_seconds or 86400
        self.botocore_config_kwargs = botocore_config_kwargs or {}
        self._client = client if client is not None else make_client(self.endpoint_url)

    @property
    def client(self):
        return self._client

    def __getattr__(self, name):
        if name.startswith("__") or name == "_client":
            raise AttributeError(name)
        return getattr(self._client, name)

    def __getstate__(self):
        return {"region_name": self.region_name, "endpoint_url": self.endpoint_url,
                "credentials": self.credentials, "role_arn": self.role_arn,
                "token_duration_seconds": self.token_duration_seconds,
                "botocore_config_kwargs": self.botocore_config_kwargs}

    def __setstate__(self, state):
        self.__init__(**state)

    def __deepcopy__(self, memo):
        return PickleableS3ClientProxy(**self.__getstate__())
