"""``s3://bucket/key`` paths (the subset of ``S3Path`` the indexing path uses).

Mirrors ``S3Path`` of the reference (``dataplug/storage/picklableS3.py:209-295``): ``from_uri``,
``from_bucket_key``, ``bucket``, ``key``, ``virtual_directory`` and ``as_uri``.  It is a plain value
type instead of a ``PurePath`` flavour subclass, which keeps it picklable and independent of
``pathlib`` internals that change between Python versions.
"""
from __future__ import annotations

import posixpath


class S3Path:
    __slots__ = ("_bucket", "_key")

    def __init__(self, bucket: str, key: str = ""):
        if not bucket or "/" in bucket:
            raise ValueError(f"invalid bucket name {bucket!r}")
        key = key.lstrip("/")
        if key:
            parts = []
            for p in key.split("/"):
                if p == "..":
                    if parts:
                        parts.pop()
                elif p not in ("", "."):
                    parts.append(p)
            key = "/".join(parts) + ("/" if key.endswith("/") and parts else "")
        self._bucket = bucket
        self._key = key

    @classmethod
    def from_uri(cls, uri: str) -> "S3Path":
        """``s3://bucket/key`` → S3Path (picklableS3.py:219-231)."""
        if not uri.startswith("s3://"):
            raise ValueError(f"Provided uri seems to be no S3 URI: {uri}")
        rest = uri[len("s3://"):]
        bucket, _, key = rest.partition("/")
        return cls(bucket, key)

    @classmethod
    def from_bucket_key(cls, bucket: str, key: str) -> "S3Path":
        """picklableS3.py:232-249."""
        return cls(bucket, key)

    @property
    def bucket(self) -> str:
        return self._bucket

    @property
    def key(self) -> str:
        return self._key

    @property
    def virtual_directory(self) -> str:
        return posixpath.dirname(self._key)

    @property
    def name(self) -> str:
        return posixpath.basename(self._key)

    def as_uri(self) -> str:
        return f"s3://{self._bucket}/{self._key}"

    def __str__(self) -> str:
        return f"/{self._bucket}/{self._key}"

    def __repr__(self) -> str:
        return f"S3Path({self.as_uri()!r})"

    def __eq__(self, other) -> bool:
        return isinstance(other, S3Path) and (self._bucket, self._key) == (other._bucket, other._key)

    def __hash__(self) -> int:
        return hash((self._bucket, self._key))

    def __getstate__(self):
        return (self._bucket, self._key)

    def __setstate__(self, state):
        self._bucket, self._key = state
