"""Plugin surface: ``CloudDataFormat``, ``CloudObjectSlice``, ``PartitioningStrategy``.

Same contract as the reference (``dataplug/entities.py:16-87``): ``@CloudDataFormat(preprocessing_function=f,
finalizer_function=g)`` on a class whose annotations/values are the attributes; ``@PartitioningStrategy(fmt)``
checks that the object is of that format.  One addition: ``batch_function`` — a format may provide a
device-batched map+reduce (all chunks of an object in one HIP launch per GPU) that produces exactly what
``finalizer_function`` over the per-chunk ``preprocessing_function`` results would; ``mapreduce_preprocessing``
uses it unless the caller asks for a joblib backend (see preprocessing/preprocess.py).
"""
from __future__ import annotations

import inspect
import logging
from enum import Enum
from pprint import pprint
from typing import TYPE_CHECKING, Callable, Optional

if TYPE_CHECKING:
    from .cloudobject import CloudObject

logger = logging.getLogger(__name__)


class PreprocessingType(Enum):
    MONOLITHIC = "monolithic"
    MAPREDUCE = "mapreduce"


class CloudDataFormat:
    def __init__(self, preprocessing_function: Optional[Callable] = None,
                 finalizer_function: Optional[Callable] = None, is_folder: bool = False,
                 batch_function: Optional[Callable] = None):
        self.co_class = None
        self.preprocessing_function = preprocessing_function
        self.finalizer_function = finalizer_function
        self.batch_function = batch_function
        self.is_folder = is_folder
        self.attrs_types = {}
        self.default_attrs = {}

    def __call__(self, cls):
        if not inspect.isclass(cls):
            raise TypeError(f"CloudObject expected to use with class type, not {type(cls)}")
        for k, t in getattr(cls, "__annotations__", {}).items():
            self.attrs_types[k] = t
        for k in dir(cls):
            if k.startswith("__") or k.endswith("__"):
                continue
            v = getattr(cls, k)
            self.attrs_types[k] = type(v)
            self.default_attrs[k] = v
        if self.co_class is not None:
            raise Exception(f"Can't overwrite decorator, now is {self.co_class}")
        self.co_class = cls
        return self

    @property
    def preprocessing_type(self) -> PreprocessingType:
        return PreprocessingType.MAPREDUCE if self.finalizer_function is not None else PreprocessingType.MONOLITHIC

    def debug(self):
        pprint({"co_class": self.co_class, "preprocessing_function": self.preprocessing_function,
                "finalizer_function": self.finalizer_function, "batch_function": self.batch_function,
                "attrs_types": self.attrs_types, "default_attrs": self.default_attrs})


class CloudObjectSlice:
    def __init__(self, range_0: Optional[int] = None, range_1: Optional[int] = None):
        self.range_0 = range_0
        self.range_1 = range_1
        self.cloud_object: Optional["CloudObject"] = None

    def get(self):
        raise NotImplementedError()


def get_slices(slices, threads: int = 16) -> list:
    """``[s.get() for s in slices]``, materialized in bulk.

    A slice class may provide ``get_many(slices, threads)`` (FASTA does: one coalesced set of ranged GETs
    for all bodies and header lines instead of 1-2 GETs per slice).  Otherwise the ``get()`` calls run on a
    thread pool (ranged GETs and copies release the GIL).  The results are those of the sequential loop;
    on the first failing slice (in slice order) its exception is raised and the slices not yet started are
    cancelled, as the loop would not have fetched them either."""
    slices = list(slices)
    if not slices:
        return []
    cls = type(slices[0])
    many = getattr(cls, "get_many", None)
    if many is not None and all(type(s) is cls for s in slices):
        return many(slices, threads=threads)
    if threads <= 1 or len(slices) <= 1:
        return [s.get() for s in slices]
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(min(threads, len(slices))) as ex:
        futs = [ex.submit(s.get) for s in slices]
        try:
            return [f.result() for f in futs]
        except BaseException:
            for f in futs:
                f.cancel()
            raise


class PartitioningStrategy:
    """Decorator for partitioning strategies (entities.py:74-87)."""

    def __init__(self, dataformat: CloudDataFormat):
        self._data_format = dataformat

    def __call__(self, func):
        def strategy_wrapper(cloud_object, *args, **kwargs):
            assert cloud_object._format_cls.co_class == self._data_format.co_class
            return func(cloud_object, *args, **kwargs)

        strategy_wrapper.__name__ = func.__name__
        strategy_wrapper.__qualname__ = func.__qualname__
        strategy_wrapper.__doc__ = func.__doc__
        strategy_wrapper.__wrapped__ = func
        return strategy_wrapper
