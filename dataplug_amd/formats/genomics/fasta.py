"""FASTA format plugin (dataplug/formats/genomics/fasta.py) with the header index built on MI355X.

Index contract (kept byte-for-byte): little-endian ``uint32`` interleaved ``[start0, end0, start1, end1, ...]``
of every header line, chunk by chunk (fasta.py:24-74).  ``start`` is the offset of a ``'>'`` that is the first
``'>'`` of its line *within its chunk* and is followed (inside the chunk) by a byte other than ``'\\n'``;
``end`` is 1 + the first ``'\\n'`` at or after ``start`` in the whole object, or the object size.  That is
what ``re.finditer(rb">.+(\\n)?")`` per chunk plus the split-header ``readline`` fix-up yields
(SURVEY.md §8(a)).  Offsets >= 2**32 raise ``OverflowError`` as numpy does in the reference, unless the
caller opts in to a uint64 index with ``extra_args={"index_dtype": "uint64"}`` (same layout, 8-byte words;
the attributes then carry ``index_dtype="uint64"`` and ``partition_chunks_strategy`` reads it back).

* ``preprocess_fasta`` — the reference's per-chunk map function (same signature); scans its chunk on GPU
  ``chunk_id % n_gpus``.
* ``merge_fasta_metadata`` — the reference's finalizer (concatenate in chunk order).
* ``batch_index_fasta`` — the default execution: every chunk in one HIP launch per GPU.
"""
from __future__ import annotations

import io
import logging
import math
import shutil
from typing import TYPE_CHECKING, List

import numpy as np

from ...entities import CloudDataFormat, CloudObjectSlice, PartitioningStrategy
from ...preprocessing.metadata import PreprocessingMetadata
from ...scan import objects as scan_objects

if TYPE_CHECKING:
    from ...cloudobject import CloudObject

logger = logging.getLogger(__name__)


INDEX_DTYPES = {"uint32": np.uint32, "uint64": np.uint64}
GET_MANY_GROUP_BYTES = 256 << 20      # slice bytes fetched per coalesced group in FASTASlice.get_many


def _index_dtype(index_dtype: str):
    """``extra_args={"index_dtype": "uint64"}`` opts in to a uint64 index (objects >= 4 GiB, where the
    reference's uint32 packing raises OverflowError, fasta.py:61-62); the default is the reference's uint32."""
    try:
        return INDEX_DTYPES[index_dtype]
    except KeyError:
        raise ValueError(f"index_dtype must be one of {sorted(INDEX_DTYPES)}, not {index_dtype!r}") from None


def _attrs(n: int, dtype) -> dict:
    a = {"num_sequences": int(n)}
    if dtype == np.uint64:       # a uint32 index keeps the reference's attributes exactly
        a["index_dtype"] = "uint64"
    return a


def preprocess_fasta(cloud_object: "CloudObject", chunk_data, chunk_id: int, chunk_size: int, num_chunks: int,
                     index_dtype: str = "uint32"):
    """Map job (fasta.py:24-63): header pairs of one chunk, scanned on the GPU."""
    dtype = _index_dtype(index_dtype)
    data = chunk_data.read()
    chunk_offset = chunk_id * chunk_size
    pairs = scan_objects.fasta_index_chunk(cloud_object, data, chunk_offset, job=chunk_id, u64=dtype == np.uint64)
    return PreprocessingMetadata(metadata=pairs.astype(dtype, copy=False).tobytes(),
                                 attributes=None if dtype == np.uint32 else {"index_dtype": index_dtype})


def merge_fasta_metadata(cloud_object: "CloudObject", chunk_metadata) -> PreprocessingMetadata:
    """Reduce job (fasta.py:66-74)."""
    ms = list(chunk_metadata)
    u64 = any((m.attributes or {}).get("index_dtype") == "uint64" for m in ms)
    dtype = np.uint64 if u64 else np.uint32
    parts = [np.frombuffer(m.metadata, dtype=dtype) for m in ms]
    num_sequences = int(sum(p.shape[0] / 2 for p in parts))
    idx = np.concatenate(parts) if parts else np.zeros(0, dtype)
    return PreprocessingMetadata(metadata=idx.tobytes(), attributes=_attrs(num_sequences, dtype))


def batch_index_fasta(cloud_object: "CloudObject", plan, chunk_size: int, num_chunks: int,
                      index_dtype: str = "uint32") -> PreprocessingMetadata:
    """Map + reduce in one go: the chunk plan scanned on the GPUs (one launch per GPU), already merged."""
    dtype = _index_dtype(index_dtype)
    pairs = scan_objects.fasta_index_object(cloud_object, plan, u64=dtype == np.uint64)
    return PreprocessingMetadata(metadata=pairs.astype(dtype, copy=False).tobytes(),
                                 attributes=_attrs(pairs.shape[0], dtype))


@CloudDataFormat(preprocessing_function=preprocess_fasta, finalizer_function=merge_fasta_metadata,
                 batch_function=batch_index_fasta)
class FASTA:
    num_sequences: int


class FASTASlice(CloudObjectSlice):
    """fasta.py:77-114: bytes [range_0, range_1) prefixed, for a slice that starts inside a sequence, with
    that sequence's header line plus `` offset=<n>``."""

    def __init__(self, offset, header, *args, **kwargs):
        self.offset = offset
        self.header = header
        super().__init__(*args, **kwargs)

    def get(self) -> bytes:
        co = self.cloud_object
        buff = io.BytesIO()
        res = co.storage.get_object(Bucket=co.path.bucket, Key=co.path.key,
                                    Range=f"bytes={self.range_0}-{self.range_1 - 1}")
        assert res["ResponseMetadata"]["HTTPStatusCode"] in (200, 206)
        if self.header is not None:
            h0, h1 = self.header
            hres = co.storage.get_object(Bucket=co.path.bucket, Key=co.path.key, Range=f"bytes={h0}-{h1 - 1}")
            line = hres["Body"].read()
            buff.write(line[:-1] + f" offset={self.offset}".encode() + b"\n")
        shutil.copyfileobj(res["Body"], buff)
        return buff.getvalue()

    @classmethod
    def get_many(cls, slices, threads: int = 16) -> list:
        """``[s.get() for s in slices]`` with batched ranged GETs: every body range and
        header line of every slice is coalesced into a few extents (neighbouring slices' bodies abut, and a
        slice's header line lies in the previous slice's body), fetched by parallel ranged GETs into one
        host buffer, and each slice is cut from it — instead of 1-2 GETs per slice.  Slices whose ranges the
        storage would not serve as plain byte ranges (empty or out-of-object) keep their own ``get()``, so
        results and errors are the reference's."""
        out = [None] * len(slices)
        by_obj = {}
        for i, s in enumerate(slices):
            co = s.cloud_object
            size = co.size
            ok = 0 <= s.range_0 < s.range_1 and s.range_0 < size
            if ok and s.header is not None:
                h0, h1 = s.header
                ok = 0 <= h0 < h1 and h0 < size
            if ok:
                by_obj.setdefault(id(co), (co, []))[1].append(i)
            else:
                out[i] = s.get()
        for co, idxs in by_obj.values():
            size = co.size
            # bounded groups of neighbouring slices: one group's extents are held at a time, so the peak host
            # memory is the results plus GET_MANY_GROUP_BYTES, not twice the requested bytes
            order = sorted(idxs, key=lambda i: slices[i].range_0)
            group, gbytes = [], 0
            for j, i in enumerate(order):
                s = slices[i]
                group.append(i)
                gbytes += min(s.range_1, size) - s.range_0
                if s.header is not None:
                    gbytes += min(s.header[1], size) - s.header[0]
                if gbytes >= GET_MANY_GROUP_BYTES or j + 1 == len(order):
                    cls._cut_group(co, slices, group, out, threads)
                    group, gbytes = [], 0
        return out

    @staticmethod
    def _cut_group(co, slices, idxs, out, threads):
        from ...storage.ranges import Extents
        size = co.size
        want = []
        for i in idxs:
            s = slices[i]
            want.append((s.range_0, min(s.range_1, size)))
            if s.header is not None:
                want.append((s.header[0], min(s.header[1], size)))
        ext = Extents(co.storage, co.path.bucket, co.path.key, want, threads=threads)
        for i in idxs:
            s = slices[i]
            body = ext.view(s.range_0, min(s.range_1, size))
            if s.header is None:
                out[i] = bytes(body)
            else:
                line = bytes(ext.view(s.header[0], min(s.header[1], size)))
                out[i] = line[:-1] + f" offset={s.offset}".encode() + b"\n" + bytes(body)
        del ext
        return out


def index_dtype_of(cloud_object: "CloudObject"):
    return np.uint64 if getattr(cloud_object.attributes, "index_dtype", "uint32") == "uint64" else np.uint32


def load_index(cloud_object: "CloudObject") -> np.ndarray:
    res = cloud_object.storage.get_object(Bucket=cloud_object.meta_path.bucket, Key=cloud_object.meta_path.key)
    return np.frombuffer(res["Body"].read(), dtype=index_dtype_of(cloud_object)).reshape(
        (cloud_object.attributes.num_sequences, 2))


@PartitioningStrategy(dataformat=FASTA)
def partition_chunks_strategy(cloud_object: "CloudObject", num_chunks: int) -> List[FASTASlice]:
    """fasta.py:117-158, same arithmetic (including its use of the index's ``end`` column)."""
    idx = load_index(cloud_object)
    wrap = 0xFFFFFFFFFFFFFFFF if idx.dtype == np.uint64 else 0xFFFFFFFF
    chunk_sz = math.ceil(cloud_object.size / num_chunks)
    ends = idx[:, 1]
    slices = []
    for i in range(num_chunks):
        r0, r1 = chunk_sz * i, chunk_sz * i + chunk_sz
        top = int(ends.searchsorted(r0))
        top = top - 1 if top > 0 else 0
        a, b = int(idx[top, 0]), int(idx[top, 1])
        if a <= r0 < b:
            r0, offset, header = a, 0, None
        else:
            offset, header = (r0 - b) & wrap, (a, b)   # index-dtype arithmetic in the reference (wraps)
        bot = int(ends.searchsorted(r0))
        if bot == idx.shape[0]:
            bot = idx.shape[0] - 1
        a2, b2 = int(idx[bot, 0]), int(idx[bot, 1])
        if a2 <= r1 < b2:
            r1 = a2
        slices.append(FASTASlice(offset=offset, header=header, range_0=r0, range_1=r1))
    return slices
