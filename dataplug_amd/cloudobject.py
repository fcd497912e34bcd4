"""``CloudObject``: the user-facing handle (dataplug/cloudobject.py:30-266), same API.

``preprocess()`` keeps the reference's semantics (cloudobject.py:215-248): assert the object exists, skip
when already preprocessed unless ``force``, create ``<bucket>.meta`` on a 404 from ``head_bucket``, then
monolithic (``chunk_size is None``) or map/reduce (``0 < chunk_size <= size``, finalizer required), then
refetch the attributes into the ``<Class>Attributes`` namedtuple.
"""
from __future__ import annotations

import logging
import pickle
from collections import namedtuple
from copy import deepcopy
from functools import partial
from typing import Any, Dict, List, Optional

from .entities import CloudDataFormat, CloudObjectSlice
from .preprocessing.preprocess import mapreduce_preprocessing, monolithic_preprocessing, use_batch_path
from .scan.objects import DEVICES_ATTR, parse_devices
from .storage.client import PickleableS3ClientProxy
from .storage.errors import ClientError
from .storage.reader import open_object
from .storage.s3path import S3Path
from .util import head_object, upload_file_with_progress

logger = logging.getLogger(__name__)


class CloudObject:
    def __init__(self, data_format: CloudDataFormat, object_path: S3Path, meta_path: S3Path, attrs_path: S3Path,
                 storage_config: Optional[Dict[str, Any]] = None, is_folder: bool = False, storage=None):
        self._obj_headers: Optional[Dict[str, Any]] = None
        self._meta_headers: Optional[Dict[str, Any]] = None
        self._attrs_headers: Optional[Dict[str, Any]] = None
        self._obj_path = object_path
        self._meta_path = meta_path
        self._attrs_path = attrs_path
        self._format_cls = data_format
        self._attrs = None
        self._is_folder = is_folder
        self._s3 = storage if storage is not None else PickleableS3ClientProxy(**(storage_config or {}))

    # ---------------------------------------------------------------- properties
    @property
    def path(self) -> S3Path:
        return self._obj_path

    @property
    def meta_path(self) -> S3Path:
        return self._meta_path

    @property
    def attrs_path(self) -> S3Path:
        return self._attrs_path

    @property
    def size(self) -> int:
        if not self._obj_headers:
            self.fetch()
        return int(self._obj_headers["ContentLength"])

    @property
    def meta_size(self) -> int:
        if self._meta_headers is None or "ContentLength" not in self._meta_headers:
            raise AttributeError()
        return int(self._meta_headers["ContentLength"])

    @property
    def storage(self):
        return self._s3

    @property
    def attributes(self) -> Any:
        return self._attrs

    @property
    def open(self):
        """``co.open("rb")`` → seekable file over ranged GETs (cloudobject.py:93-97)."""
        return partial(open_object, deepcopy(self.storage), self.path.bucket, self.path.key)

    @property
    def open_metadata(self):
        return partial(open_object, deepcopy(self.storage), self.meta_path.bucket, self.meta_path.key)

    # ---------------------------------------------------------------- constructors
    @classmethod
    def from_s3(cls, data_format: CloudDataFormat, storage_uri: str, fetch: Optional[bool] = True,
                metadata_bucket: Optional[str] = None, s3_config: Optional[Dict[str, Any]] = None) -> "CloudObject":
        obj_path = S3Path.from_uri(storage_uri)
        if metadata_bucket is None:
            metadata_bucket = obj_path.bucket + ".meta"
        co = cls(data_format, obj_path, S3Path.from_bucket_key(metadata_bucket, obj_path.key),
                 S3Path.from_bucket_key(metadata_bucket, obj_path.key + ".attrs"), s3_config, data_format.is_folder)
        if fetch:
            co.fetch()
        return co

    @classmethod
    def from_bucket_key(cls, data_format, bucket, key, fetch=True, s3_config=None) -> "CloudObject":
        co = cls(data_format, S3Path.from_bucket_key(bucket, key), S3Path.from_bucket_key(bucket + ".meta", key),
                 S3Path.from_bucket_key(bucket + ".meta", key + ".attrs"), s3_config)
        if fetch:
            co.fetch()
        return co

    @classmethod
    def new_from_file(cls, data_format, file_path, cloud_path, s3_config=None, override=False) -> "CloudObject":
        obj_path = S3Path.from_uri(cloud_path)
        co = cls(data_format, obj_path, S3Path.from_bucket_key(obj_path.bucket + ".meta", obj_path.key),
                 S3Path.from_bucket_key(obj_path.bucket + ".meta", obj_path.key + ".attrs"), s3_config)
        if co.exists():
            if not override:
                raise Exception("Object already exists")
            co.clean()
        try:
            co.storage.head_bucket(Bucket=obj_path.bucket)
        except ClientError:
            co.storage.create_bucket(Bucket=obj_path.bucket)
        upload_file_with_progress(co.storage, obj_path.bucket, obj_path.key, file_path)
        co._obj_headers = None
        return co

    # ---------------------------------------------------------------- state
    def exists(self) -> bool:
        if not self._obj_headers:
            try:
                self.fetch()
            except KeyError:
                return False
        return bool(self._obj_headers)

    def is_preprocessed(self) -> bool:
        try:
            head_object(self.storage, bucket=self._meta_path.bucket, key=self._meta_path.key)
            return True
        except KeyError:
            return False

    def fetch(self):
        if not self._obj_headers:
            if self._is_folder:
                self._obj_headers = {"Information": "folder object: no storage headers"}
            else:
                self._obj_headers, _ = head_object(self._s3, self._obj_path.bucket, self._obj_path.key)
        if not self._meta_headers:
            self._fetch_metadata()

    def _fetch_metadata(self):
        try:
            self._meta_headers, _ = head_object(self._s3, self._meta_path.bucket, self._meta_path.key)
            self._attrs_headers, _ = head_object(self._s3, self._attrs_path.bucket, self._attrs_path.key)
            res = self.storage.get_object(Bucket=self._attrs_path.bucket, Key=self._attrs_path.key)
            try:
                attrs = pickle.loads(res["Body"].read())     # written by upload_metadata (our own format)
                base = deepcopy(self._format_cls.attrs_types)
                base.update(attrs)
                nt = namedtuple(self._format_cls.co_class.__name__ + "Attributes", base.keys())
                self._attrs = nt(**base)
            except Exception as e:  # the reference logs and leaves attrs unset (cloudobject.py:203-205)
                logger.error(e)
                self._attrs = None
        except KeyError:
            self._meta_headers = None
            self._attrs = None

    def clean(self):
        self._s3.delete_object(Bucket=self._meta_path.bucket, Key=self._meta_path.key)
        self._meta_headers = None
        self.storage.delete_object(Bucket=self._attrs_path.bucket, Key=self._attrs_path.key)
        self._attrs_headers = None
        self._attrs = {}

    # ---------------------------------------------------------------- preprocessing / partitioning
    def preprocess(self, parallel_config=None, extra_args=None, chunk_size=None, force=False, debug=False):
        assert self.exists(), "Object not found in S3"
        if self.is_preprocessed() and not force:
            return
        parallel_config = parallel_config or {}
        extra_args = extra_args or {}
        try:
            meta_bucket_head = self.storage.head_bucket(Bucket=self.meta_path.bucket)
        except ClientError as error:
            if error.response["Error"]["Code"] != "404":
                raise
            meta_bucket_head = None
        if not meta_bucket_head:
            self.storage.create_bucket(Bucket=self.meta_path.bucket)

        fmt = self._format_cls
        # GPU selection: parallel_config["dataplug_devices"] (or the same key in
        # extra_args) ahead of DATAPLUG_AMD_DEVICES; it travels with the object to joblib workers
        devs = parse_devices(parallel_config.get("dataplug_devices", extra_args.get("dataplug_devices")))
        prev = getattr(self, DEVICES_ATTR, None)
        setattr(self, DEVICES_ATTR, devs)
        try:
            if chunk_size is None:
                monolithic_preprocessing(self, parallel_config, fmt.preprocessing_function, extra_args)
            else:
                assert chunk_size != 0 and chunk_size <= self.size, \
                    "Chunk size must be greater than 0 and less or equal to object size"
                assert fmt.finalizer_function is not None, "Finalizer function must be defined for mapreduce"
                batch = fmt.batch_function if use_batch_path(fmt, parallel_config) else None
                mapreduce_preprocessing(self, parallel_config, chunk_size, fmt.preprocessing_function,
                                        fmt.finalizer_function, extra_args, batch_function=batch)
        finally:
            setattr(self, DEVICES_ATTR, prev)
        self._meta_headers = None
        self.fetch()

    def get_attribute(self, key: str) -> Any:
        return getattr(self._attrs, key)

    def partition(self, strategy, *args, **kwargs) -> List[CloudObjectSlice]:
        assert self.is_preprocessed(), "Object must be preprocessed before partitioning"
        slices = strategy(self, *args, **kwargs)
        for s in slices:
            s.cloud_object = self
        return slices

    def __getitem__(self, item):
        return self._attrs.__getattribute__(item)

    def __repr__(self):
        return f"{self.__class__.__name__}<{self._format_cls.co_class.__name__}>({self.path.as_uri()})"
