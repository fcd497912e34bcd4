"""Loopback S3 endpoint (stdlib ``http.server``) over a ``MemoryStore``.

Stands in for the MinIO the reference's examples talk to (``examples/fasta_example.py:15-18``, endpoint
``http://127.0.0.1:9000``).  Path-style REST subset: HEAD/PUT bucket, HEAD/GET (``Range``)/PUT/DELETE
object, multipart uploads (POST ``?uploads``, PUT ``?partNumber&uploadId``, POST / DELETE ``?uploadId``),
ListObjectsV2, ListBuckets; user metadata as ``x-amz-meta-*``.  Unsigned.

    python -m dataplug_amd.storage.server --port 9000 [--put bucket/key=path ...] [--synth bucket/key=kind,size,seed ...]

``--synth`` materialises one of ``dataplug_amd.synth``'s seeded objects in the server process (kind ``fasta``:
tiled_fasta_host, ``csv`` / ``vcf``: tiled_csv / tiled_vcf), byte-identical to the client's own copy of the same
seed, so a benchmark's client and server need not pass gigabytes through a file.
"""
from __future__ import annotations

import argparse
import threading
import urllib.parse
import xml.etree.ElementTree as ET
from email.utils import formatdate
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Optional
from xml.sax.saxutils import escape

from .errors import ClientError
from .memory import MemoryStore, parse_range

_WRITE_BLOCK = 4 << 20


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server_version = "dataplug-amd-loopback-s3"

    def log_message(self, fmt, *args):  # quiet
        pass

    @property
    def store(self) -> MemoryStore:
        return self.server.store

    def _split(self):
        u = urllib.parse.urlsplit(self.path)
        parts = u.path.lstrip("/").split("/", 1)
        bucket = urllib.parse.unquote(parts[0]) if parts[0] else None
        key = urllib.parse.unquote(parts[1]) if len(parts) > 1 and parts[1] != "" else None
        return bucket, key, urllib.parse.parse_qs(u.query, keep_blank_values=True)

    def _send(self, status: int, body: bytes = b"", headers: Optional[dict] = None, head_only: bool = False):
        self.send_response(status)
        h = {"Content-Length": str(len(body)), "Date": formatdate(usegmt=True)}
        h.update(headers or {})
        for k, v in h.items():
            self.send_header(k, v)
        self.end_headers()
        if body and not head_only:
            self.wfile.write(body)

    def _error(self, e: ClientError, head_only: bool = False):
        code = e.response["Error"]["Code"]
        status = e.response["ResponseMetadata"]["HTTPStatusCode"]
        body = (f'<?xml version="1.0" encoding="UTF-8"?><Error><Code>{escape(code)}</Code>'
                f'<Message>{escape(e.response["Error"]["Message"])}</Message></Error>').encode()
        self._send(status, b"" if head_only else body, {"Content-Type": "application/xml"} if not head_only else {},
                   head_only=head_only)

    def _read_body(self) -> bytearray:
        n = int(self.headers.get("Content-Length") or 0)
        if self.headers.get("Transfer-Encoding", "").lower() == "chunked":
            raise ClientError("NotImplemented", "PutObject", "chunked uploads are not supported", 501)
        buf = bytearray(n)
        view = memoryview(buf)
        got = 0
        while got < n:
            r = self.rfile.readinto(view[got:])
            if not r:
                raise ClientError("IncompleteBody", "PutObject", f"{got} of {n} bytes", 400)
            got += r
        return buf                                  # (the store keeps it: no second copy of the body)

    # ---------------------------------------------------------------- verbs
    def do_HEAD(self):
        b, k, _ = self._split()
        try:
            if k is None:
                if not self.store.has_bucket(b):
                    raise ClientError("NoSuchBucket", "HeadBucket", b, 404)
                return self._send(200, head_only=True)
            o = self.store.get(b, k, "HeadObject")
            h = {"Content-Length": str(len(o.data)), "ETag": o.etag, "Accept-Ranges": "bytes",
                 "Last-Modified": formatdate(o.last_modified, usegmt=True)}
            h.update({f"x-amz-meta-{m}": v for m, v in o.metadata.items()})
            self.send_response(200)
            for hk, hv in h.items():
                self.send_header(hk, hv)
            self.end_headers()
        except ClientError as e:
            self._error(e, head_only=True)

    def do_GET(self):
        b, k, q = self._split()
        try:
            if b is None:
                names = "".join(f"<Bucket><Name>{escape(n)}</Name></Bucket>" for n in self.store.buckets())
                return self._send(200, f"<ListAllMyBucketsResult><Buckets>{names}</Buckets>"
                                       f"</ListAllMyBucketsResult>".encode(), {"Content-Type": "application/xml"})
            if k is None:
                prefix = q.get("prefix", [""])[0]
                items = "".join(f"<Contents><Key>{escape(key)}</Key><Size>{len(o.data)}</Size></Contents>"
                                for key, o in self.store.list(b, prefix))
                return self._send(200, f"<ListBucketResult><Name>{escape(b)}</Name><Prefix>{escape(prefix)}</Prefix>"
                                       f"{items}<IsTruncated>false</IsTruncated></ListBucketResult>".encode(),
                                  {"Content-Type": "application/xml"})
            o = self.store.get(b, k)
            size = len(o.data)
            r = parse_range(self.headers.get("Range"), size)
            lo, hi = r if r is not None else (0, size)
            self.send_response(206 if r is not None else 200)
            self.send_header("Content-Length", str(hi - lo))
            self.send_header("Content-Type", "binary/octet-stream")
            self.send_header("ETag", o.etag)
            self.send_header("Accept-Ranges", "bytes")
            if r is not None:
                self.send_header("Content-Range", f"bytes {lo}-{hi - 1}/{size}")
            for m, v in o.metadata.items():
                self.send_header(f"x-amz-meta-{m}", v)
            self.end_headers()
            for v in o.views(lo, hi, _WRITE_BLOCK):
                self.wfile.write(v)
        except ClientError as e:
            self._error(e)
        except (BrokenPipeError, ConnectionResetError):
            self.close_connection = True

    def do_PUT(self):
        b, k, q = self._split()
        try:
            body = self._read_body()
            if k is not None and "uploadId" in q:
                etag = self.store.upload_part(b, k, q["uploadId"][0], int(q.get("partNumber", ["0"])[0]), body,
                                              owned=True)
                return self._send(200, headers={"ETag": etag})
            if k is None:
                self.store.create_bucket(b)
                return self._send(200, headers={"Location": f"/{b}"})
            meta = {h[len("x-amz-meta-"):].lower(): v for h, v in self.headers.items()
                    if h.lower().startswith("x-amz-meta-")}
            o = self.store.put(b, k, body, meta, owned=True)
            self._send(200, headers={"ETag": o.etag})
        except ClientError as e:
            self._error(e)

    def do_POST(self):
        b, k, q = self._split()
        try:
            body = self._read_body()
            if k is None:
                raise ClientError("NotImplemented", "Post", "POST on a bucket", 501)
            if "uploads" in q:
                meta = {h[len("x-amz-meta-"):].lower(): v for h, v in self.headers.items()
                        if h.lower().startswith("x-amz-meta-")}
                uid = self.store.create_multipart(b, k, meta)
                return self._send(200, (f"<InitiateMultipartUploadResult><Bucket>{escape(b)}</Bucket><Key>{escape(k)}"
                                        f"</Key><UploadId>{uid}</UploadId></InitiateMultipartUploadResult>").encode(),
                                  {"Content-Type": "application/xml"})
            if "uploadId" in q:
                root = ET.fromstring(bytes(body))
                numbers = [int(e.text) for e in root.iter() if e.tag.endswith("PartNumber")]
                o = self.store.complete_multipart(b, k, q["uploadId"][0], numbers)
                return self._send(200, (f"<CompleteMultipartUploadResult><Bucket>{escape(b)}</Bucket><Key>{escape(k)}"
                                        f"</Key><ETag>{escape(o.etag)}</ETag></CompleteMultipartUploadResult>").encode(),
                                  {"Content-Type": "application/xml"})
            raise ClientError("NotImplemented", "Post", self.path, 501)
        except ClientError as e:
            self._error(e)

    def do_DELETE(self):
        b, k, q = self._split()
        try:
            if k is not None and "uploadId" in q:
                self.store.abort_multipart(b, k, q["uploadId"][0])
                return self._send(204)
            if k is None:
                self.store.delete_bucket(b)
            else:
                self.store.delete(b, k)
            self._send(204)
        except ClientError as e:
            self._error(e)


class _Server(ThreadingHTTPServer):
    # the listen backlog: socketserver's default of 5 drops the SYNs of a burst of parallel ranged GETs (two
    # workers x 16 GET threads per GPU), and each dropped one costs the client a 1 s retransmit
    request_queue_size = 1024


class LoopbackS3Server:
    """``with LoopbackS3Server() as srv: ... srv.endpoint_url``; serves in a daemon thread."""

    def __init__(self, store: Optional[MemoryStore] = None, host: str = "127.0.0.1", port: int = 0):
        self.store = store if store is not None else MemoryStore()
        self._httpd = _Server((host, port), _Handler)
        self._httpd.daemon_threads = True
        self._httpd.store = self.store
        self._thread: Optional[threading.Thread] = None

    @property
    def endpoint_url(self) -> str:
        host, port = self._httpd.server_address[:2]
        return f"http://{host}:{port}"

    @property
    def storage_config(self) -> dict:
        return {"endpoint_url": self.endpoint_url}

    def start(self) -> "LoopbackS3Server":
        if self._thread is None:
            self._thread = threading.Thread(target=self._httpd.serve_forever, name="loopback-s3", daemon=True)
            self._thread.start()
        return self

    def stop(self) -> None:
        if self._thread is not None:
            self._httpd.shutdown()
            self._thread.join()
            self._thread = None
        self._httpd.server_close()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


def synth_object(kind: str, size: int, seed: int):
    """The bytes of a seeded synthetic object (numpy uint8), as the client generates them."""
    from .. import synth
    if kind == "fasta":
        return synth.tiled_fasta_host(size, seed=seed)
    if kind in ("csv", "vcf"):
        obj = (synth.tiled_csv if kind == "csv" else synth.tiled_vcf)(size, seed=seed)
        return obj.bytes_range(0, size)
    raise ValueError(f"synthetic kind {kind!r}: fasta, csv or vcf")


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9000)
    ap.add_argument("--put", action="append", default=[], metavar="BUCKET/KEY=PATH")
    ap.add_argument("--bucket", action="append", default=[], help="create this (empty) bucket")
    ap.add_argument("--synth", action="append", default=[], metavar="BUCKET/KEY=KIND,SIZE,SEED")
    args = ap.parse_args(argv)
    srv = LoopbackS3Server(host=args.host, port=args.port)
    for b in args.bucket:
        srv.store.create_bucket(b)
    for spec in args.put:
        dst, _, path = spec.partition("=")
        bucket, _, key = dst.partition("/")
        srv.store.create_bucket(bucket)
        with open(path, "rb") as f:
            srv.store.put(bucket, key, f.read())
    for spec in args.synth:
        dst, _, what = spec.partition("=")
        bucket, _, key = dst.partition("/")
        kind, size, seed = what.split(",")
        srv.store.create_bucket(bucket)
        srv.store.put(bucket, key, synth_object(kind, int(size), int(seed)))
    print(f"serving {srv.endpoint_url}", flush=True)
    srv.start()
    try:
        srv._thread.join()
    except KeyboardInterrupt:
        srv.stop()


if __name__ == "__main__":
    main()
