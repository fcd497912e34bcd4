"""Map / reduce / monolithic job handlers and the metadata upload (dataplug/preprocessing/handler.py).

Storage layout kept from the reference: index at ``s3://<bucket>.meta/<key>`` (handler.py:95-100), attrs
pickle at ``<key>.attrs`` (:122-129), partials at ``<key>.chunkNNN`` (:48-56), user metadata
``{"dataplug": <version>}``, empty index object when a plugin returns no metadata (:112-119).
"""
from __future__ import annotations

import pickle

from ..util import force_delete_path
from ..version import __version__


def _check(metadata):
    if metadata.metadata is not None and metadata.metadata_file_path is not None:
        raise Exception("Choose one for object preprocessing result: metadata or metadata_file_path")


def chunk_range(size: int, chunk_id: int, chunk_size: int, num_chunks: int):
    """Byte range [r0, r1) of map job ``chunk_id`` (handler.py:36-38).

    Keeps the reference's comparison of ``chunk_size`` (not ``chunk_id``) with ``num_chunks - 1``: when it
    holds, every chunk reads to the end of the object."""
    r0 = chunk_id * chunk_size
    r1 = size if chunk_size == num_chunks - 1 else (chunk_id + 1) * chunk_size
    return r0, r1


def chunk_plan(size: int, chunk_size: int):
    """[(r0, r1)] of every map job: ``num_chunks = size // chunk_size`` (preprocess.py:38) — the tail past
    ``num_chunks * chunk_size`` is never scanned."""
    n = size // chunk_size
    return [chunk_range(size, i, chunk_size, n) for i in range(n)]


def monolith_joblib_handler(args):
    preprocessing_function, parameters = args
    co = parameters["cloud_object"]
    metadata = preprocessing_function(**parameters)
    _check(metadata)
    upload_metadata(co, metadata)


def map_joblib_handler(args):
    preprocessing_function, parameters = args
    co = parameters["cloud_object"]
    r0, r1 = chunk_range(co.size, parameters["chunk_id"], parameters["chunk_size"], parameters["num_chunks"])
    res = co.storage.get_object(Bucket=co.path.bucket, Key=co.path.key, Range=f"bytes={r0}-{r1 - 1}")
    parameters["chunk_data"] = res["Body"]
    metadata = preprocessing_function(**parameters)
    _check(metadata)
    key = f"{co.path.key}.chunk{str(parameters['chunk_id']).zfill(3)}"
    co.storage.put_object(Body=pickle.dumps(metadata), Bucket=co.meta_path.bucket, Key=key,
                          Metadata={"dataplug": __version__})
    return parameters["chunk_id"], key


def reduce_joblib_handler(args):
    finalizer_function, parameters = args
    co = parameters["cloud_object"]

    def _partials(cloud_object, partial_results):
        for _, key in partial_results:
            res = cloud_object.storage.get_object(Bucket=cloud_object.meta_path.bucket, Key=key)
            m = pickle.loads(res["Body"].read())      # our own partials (written by map_joblib_handler)
            cloud_object.storage.delete_object(Bucket=cloud_object.meta_path.bucket, Key=key)
            yield m

    metadata = finalizer_function(co, _partials(co, parameters["partial_results"]))
    _check(metadata)
    upload_metadata(co, metadata)


def upload_metadata(cloud_object, metadata):
    extra = {"Metadata": {"dataplug": __version__}}
    st = cloud_object.storage
    if metadata.metadata is not None:
        if hasattr(metadata.metadata, "read"):
            st.upload_fileobj(Fileobj=metadata.metadata, Bucket=cloud_object.meta_path.bucket,
                              Key=cloud_object.path.key, ExtraArgs=extra)
            if hasattr(metadata.metadata, "close"):
                metadata.metadata.close()
        else:
            st.put_object(Body=metadata.metadata, Bucket=cloud_object.meta_path.bucket, Key=cloud_object.path.key,
                          Metadata={"dataplug": __version__})
    if metadata.metadata_file_path is not None:
        st.upload_file(Filename=metadata.metadata_file_path, Bucket=cloud_object.meta_path.bucket,
                       Key=cloud_object.path.key, ExtraArgs=extra)
        force_delete_path(metadata.metadata_file_path)
    if metadata.metadata is None and metadata.metadata_file_path is None:
        st.put_object(Body=b"", Bucket=cloud_object.meta_path.bucket, Key=cloud_object.path.key,
                      Metadata={"dataplug": __version__})
    if metadata.attributes is not None:
        st.put_object(Body=pickle.dumps(metadata.attributes), Bucket=cloud_object._attrs_path.bucket,
                      Key=cloud_object._attrs_path.key, Metadata={"dataplug": __version__})
