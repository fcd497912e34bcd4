"""FASTA format plugin (dataplug/formats/genomics/fasta.py) with the header index built on MI355X.

Index contract (kept byte-for-byte): little-endian ``uint32`` interleaved ``[start0, end0, start1, end1, ...]``
of every header line, chunk by chunk (fasta.py:24-74).  ``start`` is the offset of a ``'>'`` that is the first
``'>'`` of its line *within its chunk* and is followed (inside the chunk) by a byte other than ``'\\n'``;
``end`` is 1 + the first ``'\\n'`` at or after ``start`` in the whole object, or the object size.  That is
what ``re.finditer(rb">.+(\\n)?")`` per chunk plus the split-header ``readline`` fix-up yields
(SURVEY.md §8(a)).  Offsets >= 2**32 raise ``OverflowError`` as numpy does in the reference.

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


def preprocess_fasta(cloud_object: "CloudObject", chunk_data, chunk_id: int, chunk_size: int, num_chunks: int):
    """Map job (fasta.py:24-63): header pairs of one chunk, scanned on the GPU."""
    data = chunk_data.read()
    chunk_offset = chunk_id * chunk_size
    pairs = scan_objects.fasta_index_chunk(cloud_object, data, chunk_offset, job=chunk_id, u64=False)
    return PreprocessingMetadata(metadata=pairs.astype(np.uint32, copy=False).tobytes())


def merge_fasta_metadata(cloud_object: "CloudObject", chunk_metadata) -> PreprocessingMetadata:
    """Reduce job (fasta.py:66-74)."""
    parts = [np.frombuffer(m.metadata, dtype=np.uint32) for m in chunk_metadata]
    num_sequences = int(sum(p.shape[0] / 2 for p in parts))
    idx = np.concatenate(parts) if parts else np.zeros(0, np.uint32)
    return PreprocessingMetadata(metadata=idx.tobytes(), attributes={"num_sequences": num_sequences})


def batch_index_fasta(cloud_object: "CloudObject", plan, chunk_size: int, num_chunks: int) -> PreprocessingMetadata:
    """Map + reduce in one go: the chunk plan scanned on the GPUs (one launch per GPU), already merged."""
    pairs = scan_objects.fasta_index_object(cloud_object, plan, u64=False)
    return PreprocessingMetadata(metadata=pairs.astype(np.uint32, copy=False).tobytes(),
                                 attributes={"num_sequences": int(pairs.shape[0])})


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


def load_index(cloud_object: "CloudObject") -> np.ndarray:
    res = cloud_object.storage.get_object(Bucket=cloud_object.meta_path.bucket, Key=cloud_object.meta_path.key)
    return np.frombuffer(res["Body"].read(), dtype=np.uint32).reshape((cloud_object.attributes.num_sequences, 2))


@PartitioningStrategy(dataformat=FASTA)
def partition_chunks_strategy(cloud_object: "CloudObject", num_chunks: int) -> List[FASTASlice]:
    """fasta.py:117-158, same arithmetic (including its use of the index's ``end`` column)."""
    idx = load_index(cloud_object)
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
            offset, header = (r0 - b) & 0xFFFFFFFF, (a, b)   # uint32 arithmetic in the reference (wraps)
        bot = int(ends.searchsorted(r0))
        if bot == idx.shape[0]:
            bot = idx.shape[0] - 1
        a2, b2 = int(idx[bot, 0]), int(idx[bot, 1])
        if a2 <= r1 < b2:
            r1 = a2
        slices.append(FASTASlice(offset=offset, header=header, range_0=r0, range_1=r1))
    return slices
