"""VCF format plugin (dataplug/formats/genomics/vcf.py) with a GPU-built newline index of the body.

``preprocess_vcf`` keeps the reference's header parse and outputs (attributes ``columns``,
``vcf_attributes``, ``body_offset``; meta object = the stripped header lines joined by '\\n',
vcf.py:19-67) and adds the offsets of every '\\n' in ``[body_offset, size)``, scanned on the GPUs in independent
parts (one or more per GPU), stored at ``<key>.lines`` (``index_format="auto"``: the u8s form, or u16b for bodies
with fewer than one newline per 128 bytes; ``_lines.store_line_index``).  ``partition_num_chunks`` gives
the reference's ranges and a ``get()`` with identical output (formulas: ``_lines.vcf_body``).
"""
from __future__ import annotations

import logging
import re
from math import ceil
from typing import TYPE_CHECKING, Dict, List, Optional, Union

from ...entities import CloudDataFormat, CloudObjectSlice, PartitioningStrategy
from ...preprocessing.metadata import PreprocessingMetadata
from .._lines import LineIndex, SliceError, index_object, slice_error, vcf_body

if TYPE_CHECKING:
    from ...cloudobject import CloudObject

logger = logging.getLogger(__name__)

_DICT_RE = re.compile(r'(\w+)=(".*?"|\w+)')


def parse_vcf_header(f):
    """(header lines, header_metadata, columns, body_offset) from a binary file object at offset 0."""
    header, meta = [], {}

    def line_of():
        raw = f.readline()
        return raw, raw.decode("utf-8").strip()

    raw, line = line_of()
    pos = len(raw)
    assert line.startswith("##fileformat=VCF"), "VCF file does not start with the correct header"
    k, v = line.replace("##", "").split("=")
    meta[k] = v
    header.append(line)
    raw, line = line_of()
    pos += len(raw)
    while line.startswith("##"):
        header.append(line)
        k, v = line.replace("##", "").split("=", 1)
        if "<" in v and ">" in v:
            v = v.strip("<").strip(">")
            d = {a: b.strip('"') for a, b in _DICT_RE.findall(v)}
            meta.setdefault(k, []).append(d)
        else:
            meta[k] = v
        raw, line = line_of()
        pos += len(raw)
    assert line.startswith("#CHROM"), "VCF file does not have the correct header"
    columns = line.replace("#", "").split("\t")
    header.append(line)
    return header, meta, columns, pos


def preprocess_vcf(cloud_object: "CloudObject", line_index: bool = True, index_format: str = "auto") -> PreprocessingMetadata:
    with cloud_object.open("rb") as f:
        header, meta, columns, body_offset = parse_vcf_header(f)
    attrs = {"columns": columns, "vcf_attributes": meta, "body_offset": body_offset}
    if line_index:
        attrs.update(index_object(cloud_object, body_offset, index_format))
    return PreprocessingMetadata(attributes=attrs, metadata="\n".join(header).encode("utf-8"))


def preprocess_vcf_gz(cloud_object: "CloudObject") -> PreprocessingMetadata:
    raise NotImplementedError("Preprocessing for VCF GZ files is not implemented yet")


@CloudDataFormat(preprocessing_function=preprocess_vcf)
class VCF:
    columns: List[str]
    vcf_attributes: Dict[str, Union[str, List[str], Dict[str, str]]]
    body_offset: int
    num_lines: int
    line_index_key: str


class VCFSlice(CloudObjectSlice):
    def __init__(self, chunk_id, num_chunks, padding, *args, body: Optional[tuple] = None,
                 error: Optional[SliceError] = None, **kwargs):
        self.chunk_id = chunk_id
        self.num_chunks = num_chunks
        self.padding = padding
        self.body = body
        self.error = error
        super().__init__(*args, **kwargs)

    def get(self) -> str:
        if self.error is not None:
            raise slice_error(self.error)
        co = self.cloud_object
        start, end = self.body
        data = b""
        if end > start:
            data = co.storage.get_object(Bucket=co.path.bucket, Key=co.path.key,
                                         Range=f"bytes={start}-{end - 1}")["Body"].read()
        header = co.storage.get_object(Bucket=co.meta_path.bucket, Key=co.meta_path.key)["Body"].read()
        return header.decode("utf-8") + "\n" + data.decode("utf-8")


@PartitioningStrategy(dataformat=VCF)
def partition_num_chunks(cloud_object: "CloudObject", num_chunks: int, padding: int = 256) -> List[VCFSlice]:
    """vcf.py:152-173."""
    size = cloud_object.size
    bo = cloud_object["body_offset"]
    chunk_size = ceil((size - bo) / num_chunks)
    lines = LineIndex.of(cloud_object)
    out = []
    for i in range(num_chunks):
        r0 = chunk_size * i + bo
        r1 = r0 + chunk_size - 1
        r0 = r0 - 1 if i != 0 else r0
        r1 = (size - 1) if r1 > size else r1
        try:
            body, err = vcf_body(lines, size, r0, r1, i, num_chunks), None
        except SliceError as e:
            body, err = None, e
        out.append(VCFSlice(range_0=r0, range_1=r1, chunk_id=i, num_chunks=num_chunks, padding=padding,
                            body=body, error=err))
    return out
