"""FASTQ.gz (dataplug/formats/genomics/fastq.py): reads = 4 lines; per-read index from the GPU scan."""
from __future__ import annotations

from math import ceil
from typing import TYPE_CHECKING, List

import numpy as np

from ...entities import PartitioningStrategy
from ..compressed.gzipped import GZipText, GZipTextSlice, _get_ranges_from_line_pairs, _line_pairs_lines_per_chunk

if TYPE_CHECKING:
    from ...cloudobject import CloudObject

FASTQGZip = GZipText


def read_pairs(total_lines: int, num_batches: int):
    """1-based [line_0, line_1) per batch (fastq.py:21-40)."""
    if (total_lines % 4) != 0:
        raise Exception("Number of lines does not correspond to FASTQ reads format!")
    num_reads = total_lines // 4
    reads_batch = ceil(num_reads / num_batches)
    rp = [(reads_batch * i, (reads_batch * i) + reads_batch) for i in range(num_batches)]
    lp = [((l0 * 4) + 1, (l1 * 4) + 1) for l0, l1 in rp]
    if lp[-1][1] > total_lines:
        lp[-1] = (lp[-1][0], total_lines + 1)
    return lp


@PartitioningStrategy(FASTQGZip)
def partition_reads_batches(cloud_object: "CloudObject", num_batches: int) -> List[GZipTextSlice]:
    """fastq.py:19-48."""
    lp = read_pairs(int(cloud_object.get_attribute("total_lines")), num_batches)
    ranges = _get_ranges_from_line_pairs(cloud_object, lp)
    return [GZipTextSlice(l0, l1, r0, r1) for (l0, l1), (r0, r1) in zip(lp, ranges)]


@PartitioningStrategy(FASTQGZip)
def partition_sequences_per_chunk(cloud_object, seq_per_chunk: int, strategy: str = "expand") -> List[GZipTextSlice]:
    """fastq.py:51-78 (keeps the reference's swapped zip order, :73-76)."""
    pairs = _line_pairs_lines_per_chunk(int(cloud_object.get_attribute("total_lines")), seq_per_chunk * 4, strategy)
    ranges = _get_ranges_from_line_pairs(cloud_object, pairs)
    return [GZipTextSlice(l0, l1, r0, r1) for (l0, l1), (r0, r1) in zip(ranges, pairs)]


def load_read_index(cloud_object) -> np.ndarray:
    """uint64 end offset (in the inflated stream) of every read, built by preprocess_gzip on the GPU."""
    key = cloud_object.get_attribute("records_key")
    res = cloud_object.storage.get_object(Bucket=cloud_object.meta_path.bucket, Key=key)
    return np.frombuffer(res["Body"].read(), dtype="<u8")
