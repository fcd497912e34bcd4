"""In-memory object store: the backing of the loopback S3 server and of ``memory://`` clients.

Objects are immutable byte buffers; a ranged read hands out a zero-copy ``memoryview`` slice.  An object made by a
multipart upload keeps its parts as they were uploaded (``Segments``: no concatenation copy at completion); a
ranged read inside one part is a view of it, one across parts a copy of the range.  Named stores
(``MemoryStore.named("x")``) are process-global so that ``memory://x`` clients created independently
(``CloudObject.open`` deep-copies its client, cloudobject.py:93-97) see the same objects.
"""
from __future__ import annotations

import bisect
import hashlib
import itertools
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, Iterator, List, Optional, Tuple

import numpy as np

from .errors import ClientError

_GIL_FREE_COPY = 1 << 20


def _own_copy(data):
    """A private copy of a PUT body: ``bytes`` when small; above 1 MiB a numpy buffer filled by ``np.copyto``, which
    copies without holding the GIL (``bytes(view)`` holds it for the whole copy, stalling every other Python thread
    of the process -- the GET threads of a streamed index build among them)."""
    try:
        view = memoryview(data).cast("B")
    except TypeError:
        return bytes(data)
    if len(view) < _GIL_FREE_COPY:
        return bytes(view)
    src = np.frombuffer(view, np.uint8)
    out = np.empty(len(src), np.uint8)
    np.copyto(out, src)
    return out


class Segments:
    """An object's bytes as the consecutive buffers of its multipart upload (read only)."""

    def __init__(self, parts: List):
        self.parts = [memoryview(p).cast("B") for p in parts if len(p)]
        self.starts = [0] + list(itertools.accumulate(len(p) for p in self.parts))

    def __len__(self) -> int:
        return self.starts[-1]

    def view(self, lo: int, hi: int):
        """Bytes [lo, hi): a view when they lie in one part, else a copy."""
        if hi <= lo:
            return memoryview(b"")
        i = bisect.bisect_right(self.starts, lo) - 1
        if hi <= self.starts[i + 1]:
            return self.parts[i][lo - self.starts[i]:hi - self.starts[i]]
        out = bytearray(hi - lo)
        p = lo
        while p < hi:
            q = min(hi, self.starts[i + 1])
            out[p - lo:q - lo] = self.parts[i][p - self.starts[i]:q - self.starts[i]]
            p, i = q, i + 1
        return memoryview(out)

    def views(self, lo: int, hi: int, block: int):
        """Views covering [lo, hi) in order, none longer than ``block`` (no copy)."""
        i = bisect.bisect_right(self.starts, lo) - 1 if hi > lo else len(self.parts)
        p = lo
        while p < hi:
            q = min(hi, self.starts[i + 1], p + block)
            yield self.parts[i][p - self.starts[i]:q - self.starts[i]]
            p = q
            if p == self.starts[i + 1]:
                i += 1

    def __bytes__(self) -> bytes:
        return b"".join(self.parts)


@dataclass
class StoredObject:
    data: object                  # bytes / bytearray / uint8 array, or Segments (a multipart upload's parts)
    metadata: Dict[str, str] = field(default_factory=dict)
    last_modified: float = field(default_factory=time.time)
    _etag: Optional[str] = None

    def view(self, lo: int, hi: int):
        """Bytes [lo, hi) of the object (a zero-copy view unless they span two multipart parts)."""
        if isinstance(self.data, Segments):
            return self.data.view(lo, hi)
        return memoryview(self.data)[lo:hi]

    def views(self, lo: int, hi: int, block: int):
        if isinstance(self.data, Segments):
            yield from self.data.views(lo, hi, block)
            return
        v = memoryview(self.data)
        for p in range(lo, hi, block):
            yield v[p:min(hi, p + block)]

    @property
    def etag(self) -> str:
        if self._etag is None:
            # md5 of a multi-GiB body is slow; a size/time tag is enough for change detection here
            h = hashlib.md5(bytes(self.view(0, len(self.data)))).hexdigest() if len(self.data) <= 1 << 20 else \
                f"{len(self.data):x}-{int(self.last_modified * 1e6):x}"
            if isinstance(self.data, Segments):
                h += f"-{len(self.data.parts)}"           # as S3 marks a multipart object's ETag
            self._etag = f'"{h}"'
        return self._etag


def parse_range(rng: Optional[str], size: int) -> Optional[Tuple[int, int]]:
    """HTTP ``Range: bytes=a-b`` (inclusive, RFC 7233) → half-open [a, b+1) clamped to ``size``.

    ``None`` means the whole object.  Raises ``ClientError("InvalidRange")`` when unsatisfiable."""
    if not rng:
        return None
    if not rng.startswith("bytes=") or "," in rng:
        raise ClientError("InvalidArgument", "GetObject", f"unsupported range {rng!r}", 400)
    a, _, b = rng[len("bytes="):].strip().partition("-")
    if a == "":                                   # suffix range: last b bytes
        n = int(b)
        if n <= 0:
            raise ClientError("InvalidRange", "GetObject", rng)
        return max(0, size - n), size
    lo = int(a)
    hi = size - 1 if b == "" else min(int(b), size - 1)
    if lo >= size or hi < lo:
        raise ClientError("InvalidRange", "GetObject", f"{rng} of {size} bytes")
    return lo, hi + 1


class MemoryStore:
    _named: Dict[str, "MemoryStore"] = {}
    _named_lock = threading.Lock()

    def __init__(self):
        self._lock = threading.RLock()
        self._buckets: Dict[str, Dict[str, StoredObject]] = {}
        self._uploads: Dict[str, Tuple[str, str, Dict[str, str], Dict[int, object]]] = {}
        self._upload_ids = itertools.count(1)

    @classmethod
    def named(cls, name: str) -> "MemoryStore":
        with cls._named_lock:
            s = cls._named.get(name)
            if s is None:
                s = cls._named[name] = cls()
            return s

    # ---------------------------------------------------------------- buckets
    def create_bucket(self, bucket: str) -> None:
        with self._lock:
            self._buckets.setdefault(bucket, {})

    def has_bucket(self, bucket: str) -> bool:
        with self._lock:
            return bucket in self._buckets

    def delete_bucket(self, bucket: str) -> None:
        with self._lock:
            b = self._buckets.get(bucket)
            if b is None:
                raise ClientError("NoSuchBucket", "DeleteBucket", bucket)
            if b:
                raise ClientError("BucketNotEmpty", "DeleteBucket", bucket)
            del self._buckets[bucket]

    def buckets(self):
        with self._lock:
            return sorted(self._buckets)

    # ---------------------------------------------------------------- objects
    def _bucket(self, bucket: str, op: str) -> Dict[str, StoredObject]:
        b = self._buckets.get(bucket)
        if b is None:
            raise ClientError("NoSuchBucket", op, bucket, 404)
        return b

    def put(self, bucket: str, key: str, data, metadata: Optional[Dict[str, str]] = None,
            owned: bool = False) -> StoredObject:
        """Store a copy of ``data``; ``owned``: a bytes / bytearray the caller hands over (kept as it is, never
        written again: the loopback server's request bodies)."""
        keep = data if owned and isinstance(data, (bytes, bytearray)) else _own_copy(data)
        obj = StoredObject(keep, dict(metadata or {}))
        with self._lock:
            self._bucket(bucket, "PutObject")[key] = obj
        return obj

    # ---------------------------------------------------------------- multipart uploads (S3 semantics)
    MIN_PART = 5 << 20                            # S3's minimum size of every part but the last

    def create_multipart(self, bucket: str, key: str, metadata: Optional[Dict[str, str]] = None) -> str:
        with self._lock:
            self._bucket(bucket, "CreateMultipartUpload")
            uid = f"mpu-{next(self._upload_ids):08d}"
            self._uploads[uid] = (bucket, key, dict(metadata or {}), {})
        return uid

    def _upload(self, bucket: str, key: str, uid: str, op: str):
        u = self._uploads.get(uid)
        if u is None or u[0] != bucket or u[1] != key:
            raise ClientError("NoSuchUpload", op, f"{bucket}/{key} upload {uid}", 404)
        return u

    def upload_part(self, bucket: str, key: str, uid: str, number: int, data, owned: bool = False) -> str:
        """Store part ``number`` (1..10000) of an upload, a copy of ``data`` unless ``owned``; returns its ETag."""
        if not 1 <= int(number) <= 10000:
            raise ClientError("InvalidArgument", "UploadPart", f"part number {number}", 400)
        keep = data if owned and isinstance(data, (bytes, bytearray)) else _own_copy(data)
        with self._lock:
            self._upload(bucket, key, uid, "UploadPart")[3][int(number)] = keep
        return f'"{hashlib.md5(memoryview(keep)[:1 << 16]).hexdigest()}-{len(keep):x}"'

    def complete_multipart(self, bucket: str, key: str, uid: str, numbers: List[int]) -> StoredObject:
        """The object made of the listed parts in ascending order (every one but the last >= MIN_PART)."""
        with self._lock:
            _, _, meta, parts = self._upload(bucket, key, uid, "CompleteMultipartUpload")
            if not numbers or list(numbers) != sorted(set(numbers)) or any(n not in parts for n in numbers):
                raise ClientError("InvalidPart", "CompleteMultipartUpload", f"parts {list(numbers)[:8]}", 400)
            if any(len(parts[n]) < self.MIN_PART for n in numbers[:-1]):
                raise ClientError("EntityTooSmall", "CompleteMultipartUpload", "a part below 5 MiB", 400)
            obj = StoredObject(Segments([parts[n] for n in numbers]), meta)
            self._bucket(bucket, "CompleteMultipartUpload")[key] = obj
            del self._uploads[uid]
        return obj

    def abort_multipart(self, bucket: str, key: str, uid: str) -> None:
        with self._lock:
            self._upload(bucket, key, uid, "AbortMultipartUpload")
            del self._uploads[uid]

    def get(self, bucket: str, key: str, op: str = "GetObject") -> StoredObject:
        with self._lock:
            obj = self._bucket(bucket, op).get(key)
        if obj is None:
            raise ClientError("NoSuchKey", op, f"{bucket}/{key}", 404)
        return obj

    def delete(self, bucket: str, key: str) -> None:
        with self._lock:
            self._bucket(bucket, "DeleteObject").pop(key, None)

    def list(self, bucket: str, prefix: str = "") -> Iterator[Tuple[str, StoredObject]]:
        with self._lock:
            items = sorted(self._bucket(bucket, "ListObjectsV2").items())
        return ((k, o) for k, o in items if k.startswith(prefix))
