"""Monolithic and map/reduce preprocessing drivers (dataplug/preprocessing/preprocess.py).

``mapreduce_preprocessing`` builds the same job list as the reference (``num_chunks = size // chunk_size``,
jobs sorted by ``chunk_id`` before the reduce).  Execution:

* the format's ``batch_function`` (device-batched: every chunk of the object scanned by one HIP launch per
  GPU, outputs already concatenated in chunk order) — the default, used when ``parallel_config`` names no
  joblib ``backend``;
* otherwise joblib with the caller's ``parallel_config``, one map job per chunk (each job's plugin call
  runs on GPU ``chunk_id % n_gpus``), then the reduce job — the reference's execution shape.

Both end in the same stored index and attributes.
"""
from __future__ import annotations

import inspect
import os

import joblib

from .handler import chunk_plan, map_joblib_handler, monolith_joblib_handler, reduce_joblib_handler, upload_metadata


def monolithic_preprocessing(cloud_object, parallel_config, preprocessing_function, extra_args):
    sig = inspect.signature(preprocessing_function).parameters
    if "cloud_object" not in sig:
        raise Exception("Preprocessing function must have cloud_object as a parameter")
    args = {"cloud_object": cloud_object}
    for a in sig:
        if a not in args and a in extra_args:
            args[a] = extra_args[a]
    with joblib.parallel_config(**_joblib_config(parallel_config)):
        list(joblib.Parallel()([joblib.delayed(monolith_joblib_handler)((preprocessing_function, args))]))


def _joblib_config(parallel_config):
    return {k: v for k, v in (parallel_config or {}).items() if not k.startswith("dataplug_")}


def use_batch_path(fmt, parallel_config) -> bool:
    if getattr(fmt, "batch_function", None) is None:
        return False
    if os.environ.get("DATAPLUG_AMD_BATCH", "1") == "0":
        return False
    pc = parallel_config or {}
    if "dataplug_batch" in pc:
        return bool(pc["dataplug_batch"])
    return "backend" not in pc


def mapreduce_preprocessing(cloud_object, parallel_config, chunk_size, preprocessing_function, finalizer_function,
                            extra_args, batch_function=None):
    sig = inspect.signature(preprocessing_function).parameters
    if not {"chunk_data", "chunk_id", "chunk_size", "num_chunks"}.issubset(sig.keys()):
        raise Exception("Preprocessing function must have (chunk_data, chunk_id, chunk_size, num_chunks) as parameters")
    num_chunks = cloud_object.size // chunk_size
    extras = {}
    for a, prm in sig.items():
        if a not in ("cloud_object", "chunk_id", "chunk_size", "num_chunks", "chunk_data"):
            if a not in extra_args and prm.default is not inspect.Parameter.empty:
                continue                     # optional plugin keyword (e.g. FASTA index_dtype): its default
            extras[a] = extra_args[a]        # KeyError like the reference when an extra arg is missing

    if batch_function is not None:
        metadata = batch_function(cloud_object, chunk_plan(cloud_object.size, chunk_size), chunk_size=chunk_size,
                                  num_chunks=num_chunks, **extras)
        if metadata.metadata is not None and metadata.metadata_file_path is not None:
            raise Exception("Choose one for object preprocessing result: metadata or metadata_file_path")
        upload_metadata(cloud_object, metadata)
        return

    jobs = []
    for chunk_id in range(num_chunks):
        args = {"cloud_object": cloud_object, "chunk_id": chunk_id, "chunk_size": chunk_size,
                "num_chunks": num_chunks, "chunk_data": None}
        args.update(extras)
        jobs.append(args)
    with joblib.parallel_config(**_joblib_config(parallel_config)):
        jl = joblib.Parallel()
        partial_results = list(jl([joblib.delayed(map_joblib_handler)((preprocessing_function, j)) for j in jobs]))
        partial_results.sort(key=lambda x: x[0])
        args = {"cloud_object": cloud_object, "partial_results": partial_results}
        list(jl([joblib.delayed(reduce_joblib_handler)((finalizer_function, args))]))
