"""CSV format plugin (dataplug/formats/generic/csv.py) with a GPU-built newline index.

``preprocess_csv`` keeps the reference's attributes (``columns``/``dtypes`` from the first 20 lines,
csv.py:20-36) and additionally stores the sorted offsets of every ``'\\n'`` (scanned on the GPUs) at
``<key>.lines`` in the meta bucket (attributes ``num_lines``, ``line_index_key``, ``line_index_dtype``; with
``index_format="auto"`` the u8s form, or u16b for objects with fewer than one newline per 128 bytes).  The meta
object itself stays empty, as in the reference.  The partition strategies produce the reference's
``range_0``/``range_1`` and a ``get()`` with identical output, resolved from the index instead of a
padded Python scan per slice (the reference's formulas: ``_lines.csv_body``).
"""
from __future__ import annotations

import io
import logging
from math import ceil
from typing import TYPE_CHECKING, List, Optional

from ...entities import CloudDataFormat, CloudObjectSlice, PartitioningStrategy
from ...preprocessing.metadata import PreprocessingMetadata
from .._lines import LineIndex, SliceError, csv_body, index_object, slice_error

if TYPE_CHECKING:
    from ...cloudobject import CloudObject

logger = logging.getLogger(__name__)


def preprocess_csv(cloud_object: "CloudObject", separator: str = ",", line_index: bool = True,
                   index_format: str = "auto") -> PreprocessingMetadata:
    import pandas as pd

    top = []
    with cloud_object.open("r") as f:
        for _ in range(20):
            top.append(f.readline().strip())
    df = pd.read_csv(io.StringIO("\n".join(top)), sep=separator)
    attrs = {"columns": df.columns.tolist(), "dtypes": df.dtypes.tolist()}
    if line_index:
        attrs.update(index_object(cloud_object, 0, index_format))
    return PreprocessingMetadata(attributes=attrs)


@CloudDataFormat(preprocessing_function=preprocess_csv)
class CSV:
    columns: List[str]
    dtypes: List[str]
    num_lines: int
    line_index_key: str


class CSVSlice(CloudObjectSlice):
    def __init__(self, chunk_id, num_chunks, padding, *args, body: Optional[tuple] = None,
                 error: Optional[SliceError] = None, **kwargs):
        self.chunk_id = chunk_id
        self.num_chunks = num_chunks
        self.padding = padding
        self.body = body            # object bytes [start, end) this slice returns
        self.error = error
        super().__init__(*args, **kwargs)

    def get_bytes(self) -> bytes:
        if self.error is not None:
            raise slice_error(self.error)
        co = self.cloud_object
        start, end = self.body
        data = b""
        if end > start:
            data = co.storage.get_object(Bucket=co.path.bucket, Key=co.path.key,
                                         Range=f"bytes={start}-{end - 1}")["Body"].read()
        if self.range_0 != 0:
            data = (",".join(co.attributes.columns) + "\n").encode("utf-8") + data
        return data

    def get(self) -> str:
        return self.get_bytes().decode("utf-8")

    def get_as_pandas(self):
        import pandas as pd
        return pd.read_csv(io.StringIO(self.get()))


def _slices(cloud_object, chunk_size: int, num_chunks: int, padding: int) -> List[CSVSlice]:
    size = cloud_object.size
    lines = LineIndex.of(cloud_object)
    out = []
    for i in range(num_chunks):
        r0 = chunk_size * i
        r0 = r0 - 1 if r0 > 0 else r0
        r1 = chunk_size * i + chunk_size
        r1 = size if r1 > size else r1 + padding
        try:
            body, err = csv_body(lines, size, r0, r1, i, num_chunks, padding), None
        except SliceError as e:
            body, err = None, e
        out.append(CSVSlice(range_0=r0, range_1=r1, chunk_id=i, num_chunks=num_chunks, padding=padding,
                            body=body, error=err))
    return out


@PartitioningStrategy(dataformat=CSV)
def partition_chunk_size(cloud_object: "CloudObject", chunk_size: int, padding: int = 256) -> List[CSVSlice]:
    """csv.py:112-129."""
    assert chunk_size <= cloud_object.size, "Chunk size must be smaller than the file size"
    return _slices(cloud_object, chunk_size, ceil(cloud_object.size / chunk_size), padding)


@PartitioningStrategy(dataformat=CSV)
def partition_num_chunks(cloud_object: "CloudObject", num_chunks: int, padding: int = 256) -> List[CSVSlice]:
    """csv.py:132-148."""
    return _slices(cloud_object, ceil(cloud_object.size / num_chunks), num_chunks, padding)
