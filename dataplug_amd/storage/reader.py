"""Seekable read-only file over ranged GETs: what ``CloudObject.open("rb"|"r")`` returns.

The reference returns ``smart_open.open`` over its client (cloudobject.py:93-97); its callers on the
indexing path use ``seek``/``readline``/``tell`` (fasta.py:49-53) and text ``readline`` (csv.py:20-25,
vcf.py:19-52).  ``io.BufferedReader`` over a ``RawIOBase`` that issues one ranged GET per refill gives the
same surface.
"""
from __future__ import annotations

import io
from typing import Optional


class RangedReader(io.RawIOBase):
    def __init__(self, client, bucket: str, key: str, size: Optional[int] = None):
        self._client = client
        self._bucket = bucket
        self._key = key
        self._size = int(size) if size is not None else int(client.head_object(Bucket=bucket, Key=key)["ContentLength"])
        self._pos = 0

    @property
    def size(self) -> int:
        return self._size

    def readable(self) -> bool:
        return True

    def seekable(self) -> bool:
        return True

    def tell(self) -> int:
        return self._pos

    def seek(self, offset: int, whence: int = io.SEEK_SET) -> int:
        base = {io.SEEK_SET: 0, io.SEEK_CUR: self._pos, io.SEEK_END: self._size}[whence]
        pos = base + offset
        if pos < 0:
            raise ValueError(f"negative seek position {pos}")
        self._pos = pos
        return pos

    def readinto(self, b) -> int:
        n = min(len(b), self._size - self._pos)
        if n <= 0:
            return 0
        res = self._client.get_object(Bucket=self._bucket, Key=self._key, Range=f"bytes={self._pos}-{self._pos + n - 1}")
        body = res["Body"]
        view = memoryview(b).cast("B")
        got = 0
        with body:
            while got < n:
                r = body.readinto(view[got:n])
                if not r:
                    break
                got += r
        self._pos += got
        return got


def open_object(client, bucket: str, key: str, mode: str = "rb", buffer_size: int = 1 << 18,
                encoding: str = "utf-8", size: Optional[int] = None):
    if any(c in mode for c in "wax+"):
        raise ValueError(f"read-only object file, mode {mode!r}")
    raw = RangedReader(client, bucket, key, size)
    buf = io.BufferedReader(raw, buffer_size=buffer_size)
    if "b" in mode:
        return buf
    return io.TextIOWrapper(buf, encoding=encoding)
