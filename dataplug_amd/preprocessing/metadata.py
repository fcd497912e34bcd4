"""``PreprocessingMetadata`` (dataplug/preprocessing/metadata.py:13-17): what a plugin returns."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, BinaryIO, Dict, Optional, Union


@dataclass
class PreprocessingMetadata:
    metadata: Optional[Union[BinaryIO, bytes]] = None
    metadata_file_path: Optional[str] = None
    attributes: Optional[Dict[str, Any]] = None
