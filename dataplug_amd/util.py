"""Helpers of the reference's ``dataplug/util.py`` used on the indexing path."""
from __future__ import annotations

import logging
import os
import re
import shutil

from .storage.errors import ClientError

logger = logging.getLogger(__name__)

S3_PATH_REGEX = re.compile(r"^\w+://.+/.+$")


def setup_logging(level=logging.INFO):
    root = logging.getLogger("dataplug_amd")
    root.setLevel(level)
    ch = logging.StreamHandler()
    ch.setLevel(logging.DEBUG)
    ch.setFormatter(logging.Formatter("[%(asctime)s] %(levelname)s [%(name)s.%(funcName)s:%(lineno)d] %(message)s"))
    root.addHandler(ch)


def split_s3path_string(path: str):
    if not S3_PATH_REGEX.fullmatch(path):
        raise ValueError(f"Path must satisfy regex {S3_PATH_REGEX}")
    bucket, key = path.replace("s3://", "").split("/", 1)
    return bucket, key


def force_delete_path(path):
    if path and os.path.exists(path):
        if os.path.isfile(path):
            os.remove(path)
        elif os.path.isdir(path):
            shutil.rmtree(path)


def head_object(s3client, bucket, key):
    """(headers, user metadata); a 404 becomes ``KeyError`` (util.py:46-60)."""
    try:
        res = dict(s3client.head_object(Bucket=bucket, Key=key))
    except ClientError as e:
        if e.response["Error"]["Code"] == "404":
            raise KeyError(f"{bucket}/{key}") from None
        raise
    res.pop("ResponseMetadata", None)
    meta = res.pop("Metadata", {}) or {}
    return res, dict(meta)


def upload_file_with_progress(s3client, bucket, key, filename):
    with open(filename, "rb") as f:
        s3client.upload_fileobj(f, bucket, key)
