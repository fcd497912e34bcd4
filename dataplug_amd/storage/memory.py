"""In-memory object store: the backing of the loopback S3 server and of ``memory://`` clients.

Objects are immutable ``bytes``; a ranged read hands out a zero-copy ``memoryview`` slice.  Named stores
(``MemoryStore.named("x")``) are process-global so that ``memory://x`` clients created independently
(``CloudObject.open`` deep-copies its client, cloudobject.py:93-97) see the same objects.
"""
from __future__ import annotations

import hashlib
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, Iterator, Optional, Tuple

from .errors import ClientError


@dataclass
class StoredObject:
    data: bytes
    metadata: Dict[str, str] = field(default_factory=dict)
    last_modified: float = field(default_factory=time.time)
    _etag: Optional[str] = None

    @property
    def etag(self) -> str:
        if self._etag is None:
            # md5 of a multi-GiB body is slow; a size/time tag is enough for change detection here
            h = hashlib.md5(self.data[:1 << 20]).hexdigest() if len(self.data) <= 1 << 20 else \
                f"{len(self.data):x}-{int(self.last_modified * 1e6):x}"
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
        keep = data if owned and isinstance(data, (bytes, bytearray)) else bytes(data)
        obj = StoredObject(keep, dict(metadata or {}))
        with self._lock:
            self._bucket(bucket, "PutObject")[key] = obj
        return obj

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
