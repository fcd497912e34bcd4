"""Generate the committed golden fixtures by running the REFERENCE dataplug in this container.

Run here only (needs /root/reference, which never travels to the GPU box):

    python tests/golden/make_golden.py

How the reference is run: boto3/botocore/smart_open are not installed, so tiny
stand-in modules are put in ``sys.modules`` before ``import dataplug``; a ``CloudObject`` is built
with ``object.__new__`` (its constructor calls STS) and given an in-memory S3 fake whose ranged GET
is INCLUSIVE like S3.  ``co.preprocess(chunk_size=...)`` then runs the reference's own
``mapreduce_preprocessing`` -> ``map_joblib_handler`` -> ``preprocess_fasta`` -> ``merge_fasta_metadata``
-> ``upload_metadata`` unchanged, and slices come from the reference's own ``partition_*`` + ``get()``.

Outputs (data only: inputs + the reference's outputs):
  fasta_cases.npz      fuzz + sample + synthetic FASTA inputs, chunk sizes, expected uint32 indexes
  fasta_slices.json    partition_chunks_strategy slices (+ get() bytes for the sample object)
  csv_slices.json      CSV attrs + partition_num_chunks / partition_chunk_size get() outputs (cities.csv,
                       synthetic, and rows longer than the 256 B padding: the buffer-expansion path)
  vcf_slices.json      VCF attrs + header meta + partition_num_chunks get() outputs (sample.vcf, synthetic,
                       and rows longer than the padding: the range-expansion path)
  fastq_batches.json   partition_reads_batches line pairs (gztool absent: parity unpinned beyond these)
"""
from __future__ import annotations

import base64
import io
import json
import math
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from dataplug_amd import synth  # noqa: E402


# --------------------------------------------------------------------------- stand-in modules
class ClientError(Exception):
    def __init__(self, code):
        super().__init__(code)
        self.response = {"Error": {"Code": str(code)}}


def _install_stubs(store):
    boto3 = types.ModuleType("boto3")
    boto3.client = lambda *a, **k: None
    s3 = types.ModuleType("boto3.s3")
    transfer = types.ModuleType("boto3.s3.transfer")
    transfer.TransferConfig = lambda **k: dict(k)
    boto3.s3 = s3
    s3.transfer = transfer
    botocore = types.ModuleType("botocore")
    exc = types.ModuleType("botocore.exceptions")
    exc.ClientError = ClientError
    client = types.ModuleType("botocore.client")
    client.Config = lambda **k: dict(k)
    resp = types.ModuleType("botocore.response")
    resp.StreamingBody = io.BytesIO
    botocore.exceptions, botocore.client, botocore.response = exc, client, resp
    smart_open = types.ModuleType("smart_open")

    def _open(uri, mode="rb", transport_params=None):
        bucket, key = uri[len("s3://"):].split("/", 1)
        raw = io.BytesIO(store[bucket][key])
        return raw if "b" in mode else io.TextIOWrapper(raw, encoding="utf-8", newline="")

    smart_open.open = _open
    smart_open.smart_open = _open
    for name, mod in {"boto3": boto3, "boto3.s3": s3, "boto3.s3.transfer": transfer, "botocore": botocore,
                      "botocore.exceptions": exc, "botocore.client": client, "botocore.response": resp,
                      "smart_open": smart_open}.items():
        sys.modules[name] = mod


class FakeS3:
    """In-memory S3 with inclusive ``Range: bytes=a-b`` (S3 semantics, unlike filesystem.py:64-69); a range
    starting at or past the object's end fails with InvalidRange (HTTP 416), as on S3."""

    def __init__(self, store):
        self.store = store

    def __deepcopy__(self, memo):
        return self

    def _obj(self, Bucket, Key):
        try:
            return self.store[Bucket][Key]
        except KeyError:
            raise ClientError(404)

    def head_object(self, Bucket, Key):
        d = self._obj(Bucket, Key)
        return {"ResponseMetadata": {"HTTPStatusCode": 200}, "ContentLength": len(d), "Metadata": {}}

    def head_bucket(self, Bucket):
        if Bucket not in self.store:
            raise ClientError(404)
        return {"ResponseMetadata": {"HTTPStatusCode": 200}}

    def create_bucket(self, Bucket):
        self.store.setdefault(Bucket, {})
        return {"ResponseMetadata": {"HTTPStatusCode": 200}}

    def get_object(self, Bucket, Key, Range=None):
        d = self._obj(Bucket, Key)
        code = 200
        if Range is not None:
            a, b = Range[len("bytes="):].split("-")
            if int(a) >= len(d):                 # S3: a range starting at or past the end -> 416
                raise ClientError("InvalidRange")
            d = d[int(a):int(b) + 1]
            code = 206
        return {"Body": io.BytesIO(d), "ResponseMetadata": {"HTTPStatusCode": code}}

    def put_object(self, Body, Bucket, Key, Metadata=None):
        self.store.setdefault(Bucket, {})[Key] = Body if isinstance(Body, bytes) else Body.read()
        return {"ResponseMetadata": {"HTTPStatusCode": 200}}

    def upload_fileobj(self, Fileobj, Bucket, Key, ExtraArgs=None, Config=None):
        self.store.setdefault(Bucket, {})[Key] = Fileobj.read()

    def delete_object(self, Bucket, Key):
        self.store.get(Bucket, {}).pop(Key, None)
        return {"ResponseMetadata": {"HTTPStatusCode": 204}}


STORE: dict = {}
_install_stubs(STORE)
sys.path.insert(0, REF)
import dataplug  # noqa: E402
from dataplug.cloudobject import CloudObject  # noqa: E402
from dataplug.storage.picklableS3 import S3Path  # noqa: E402
from dataplug.formats.genomics import fasta as ref_fasta  # noqa: E402
from dataplug.formats.generic import csv as ref_csv  # noqa: E402
from dataplug.formats.genomics import vcf as ref_vcf  # noqa: E402
from dataplug.formats.genomics import fastq as ref_fastq  # noqa: E402

S3 = FakeS3(STORE)


def make_co(fmt, bucket, key, data: bytes):
    STORE.setdefault(bucket, {})[key] = data
    for k in (key, key + ".attrs"):
        STORE.get(bucket + ".meta", {}).pop(k, None)
    co = object.__new__(CloudObject)
    co._obj_headers = co._meta_headers = co._attrs_headers = None
    co._obj_path = S3Path.from_bucket_key(bucket, key)
    co._meta_path = S3Path.from_bucket_key(bucket + ".meta", key)
    co._attrs_path = S3Path.from_bucket_key(bucket + ".meta", key + ".attrs")
    co._format_cls = fmt
    co._attrs = None
    co._is_folder = False
    co._s3 = S3
    co.fetch()
    return co


# --------------------------------------------------------------------------- FASTA
def ref_fasta_index(data: bytes, chunk_size: int):
    """Reference co.preprocess(chunk_size) -> (index bytes or None, num_sequences or error name)."""
    co = make_co(ref_fasta.FASTA, "genomics", "obj.fasta", data)
    try:
        co.preprocess(chunk_size=chunk_size, force=True)
    except OverflowError:
        return None, "OverflowError"
    meta = STORE["genomics.meta"]["obj.fasta"]
    return meta, co.attributes.num_sequences


def fasta_cases():
    rng = np.random.default_rng(20251015)
    inputs, chunk_sizes, kinds, expected, exp_off, nseq = [], [], [], [], [0], []

    def add(data: bytes, cs: int, kind: str):
        meta, n = ref_fasta_index(data, cs)
        assert meta is not None, kind
        inputs.append(data)
        chunk_sizes.append(cs)
        kinds.append(kind)
        arr = np.frombuffer(meta, np.uint32)
        expected.append(arr)
        exp_off.append(exp_off[-1] + len(arr))
        nseq.append(n)

    sample = open(os.path.join(REF, "examples/sample_data/fasta_sample.fasta"), "rb").read()
    for cs in [math.ceil(len(sample) / 4), len(sample), 1, 7, 60, 61, 100, 255, 534, 1000, len(sample) // 2]:
        add(sample, cs, "sample")
    # adversarial fuzz over a tiny alphabet; tail-drop, last-byte '>', cs == n-1, '\r', '>>', '>\n', mid-line '>'
    alphabets = [b">\nA", b">\nAC\r ", b">>\n\nAAAAAA", b">\nACGTACGTACGT"]
    for i in range(1500):
        alpha = np.frombuffer(alphabets[i % len(alphabets)], np.uint8)
        size = int(rng.integers(1, 200 if i % 3 else 40))
        data = bytes(alpha[rng.integers(0, len(alpha), size)])
        if i % 5 == 0:
            cs = max(1, int(math.isqrt(size)) - 1)  # often hits chunk_size == num_chunks - 1
        else:
            cs = int(rng.integers(1, size + 1))
        add(data, cs, "fuzz")
    # explicit chunk_size == num_chunks-1 quirk cases (every chunk reads to EOF)
    for size, cs in [(12, 3), (20, 4), (30, 5), (7, 2), (42, 6)]:
        alpha = np.frombuffer(b">\nAC", np.uint8)
        data = bytes(alpha[rng.integers(0, 4, size)])
        assert size // cs == cs + 1
        add(data, cs, "quirk_cs_eq_n_minus_1")
    # synthetic FASTA (seeded, regenerated in tests from synth.fasta; only the index is large)
    syn = []
    for seed, size in [(1, 1 << 20), (2, (1 << 20) + 12345), (3, 3 << 20)]:
        data = synth.fasta(size, seed)
        for div in [1, 4, 7, 64]:
            cs = math.ceil(size / div)
            meta, n = ref_fasta_index(bytes(data), cs)
            syn.append({"seed": seed, "size": size, "sha256": synth.sha256(data), "chunk_size": cs,
                        "num_sequences": n, "index": np.frombuffer(meta, np.uint32)})
    return inputs, chunk_sizes, kinds, expected, exp_off, nseq, syn


def fasta_slices():
    out = []
    sample = open(os.path.join(REF, "examples/sample_data/fasta_sample.fasta"), "rb").read()
    objs = [("sample", sample, [math.ceil(len(sample) / 4)], [1, 2, 3, 5, 8, 13])]
    objs.append(("synth1", bytes(synth.fasta(1 << 18, 11)), [1 << 16], [1, 3, 8, 50]))
    for name, data, css, nchunks in objs:
        for cs in css:
            co = make_co(ref_fasta.FASTA, "genomics", name, data)
            co.preprocess(chunk_size=cs, force=True)
            for n in nchunks:
                slices = co.partition(ref_fasta.partition_chunks_strategy, num_chunks=n)
                rec = {"object": name, "chunk_size": cs, "num_chunks": n,
                       "slices": [[int(s.offset), None if s.header is None else [int(x) for x in s.header],
                                   int(s.range_0), int(s.range_1)] for s in slices]}
                if name == "sample":
                    rec["get"] = [base64.b64encode(s.get()).decode() for s in slices]
                out.append(rec)
    return out


# --------------------------------------------------------------------------- CSV / VCF
def _get(s):
    """slice.get() or the name of the exception the reference raises."""
    try:
        return s.get()
    except Exception as e:  # noqa: BLE001
        return {"error": type(e).__name__}


def csv_slices():
    cities = open(os.path.join(REF, "examples/sample_data/cities.csv"), "rb").read()
    out = {"objects": []}
    for name, data in [("cities", cities), ("synth_csv", bytes(synth.csv(1 << 16, 5))),
                       ("wide_csv", bytes(synth.csv_wide(1 << 16, 5)))]:
        co = make_co(ref_csv.CSV, "dataplug", name, data)
        co.preprocess(force=True)
        rec = {"object": name, "sha256": synth.sha256(np.frombuffer(data, np.uint8)),
               "columns": list(co.attributes.columns), "dtypes": [str(d) for d in co.attributes.dtypes],
               "num_chunks": {}, "chunk_size": {}}
        for n in [1, 2, 3, 5, 25, 100]:
            sl = co.partition(ref_csv.partition_num_chunks, num_chunks=n)
            rec["num_chunks"][str(n)] = [[s.range_0, s.range_1, _get(s)] for s in sl]
        for cs in [100, 1000, len(data) // 3]:
            sl = co.partition(ref_csv.partition_chunk_size, chunk_size=cs)
            rec["chunk_size"][str(cs)] = [[s.range_0, s.range_1, _get(s)] for s in sl]
        out["objects"].append(rec)
    return out


def vcf_slices():
    sample = open(os.path.join(REF, "examples/sample_data/sample.vcf"), "rb").read()
    out = {"objects": []}
    for name, data in [("sample", sample), ("synth_vcf", bytes(synth.vcf(1 << 16, 6))),
                       ("wide_vcf", bytes(synth.vcf_wide(1 << 16, 6)))]:
        co = make_co(ref_vcf.VCF, "dataplug", name, data)
        co.preprocess(force=True)
        rec = {"object": name, "sha256": synth.sha256(np.frombuffer(data, np.uint8)),
               "columns": list(co.attributes.columns), "vcf_attributes": co.attributes.vcf_attributes,
               "body_offset": co.attributes.body_offset,
               "meta": STORE["dataplug.meta"][name].decode(), "num_chunks": {}}
        for n in [1, 2, 3, 4, 7, 16, 33]:
            sl = co.partition(ref_vcf.partition_num_chunks, num_chunks=n)
            rec["num_chunks"][str(n)] = [[s.range_0, s.range_1, _get(s)] for s in sl]
        out["objects"].append(rec)
    return out


# --------------------------------------------------------------------------- FASTQ (read batching only)
class _Attrs:
    def __init__(self, total_lines):
        self.total_lines = total_lines


def fastq_batches():
    captured = []

    def fake_ranges(co, pairs):
        captured.append([list(map(int, p)) for p in pairs])
        return [(i, i + 1) for i in range(len(pairs))]

    ref_fastq._get_ranges_from_line_pairs = fake_ranges
    out = []
    for total_lines in [4, 40, 400, 4000, 4 * 12345]:
        for nb in [1, 2, 3, 7, 10]:
            if nb * 1 > total_lines // 4:
                continue
            co = object.__new__(CloudObject)
            co._format_cls = ref_fastq.FASTQGZip
            co._attrs = types.SimpleNamespace(total_lines=total_lines)
            captured.clear()
            slices = ref_fastq.partition_reads_batches(co, num_batches=nb)
            out.append({"total_lines": total_lines, "num_batches": nb,
                        "line_pairs": [[s.line_0, s.line_1] for s in slices]})
    # the error branch: total_lines not a multiple of 4
    co = object.__new__(CloudObject)
    co._format_cls = ref_fastq.FASTQGZip
    co._attrs = types.SimpleNamespace(total_lines=10)
    try:
        ref_fastq.partition_reads_batches(co, num_batches=2)
        err = None
    except Exception as e:  # noqa: BLE001
        err = str(e)
    return {"cases": out, "non_multiple_of_4_error": err}


def main():
    inputs, cs, kinds, exp, exp_off, nseq, syn = fasta_cases()
    lens = np.array([len(x) for x in inputs], np.int64)
    np.savez_compressed(
        os.path.join(HERE, "fasta_cases.npz"),
        data=np.frombuffer(b"".join(inputs), np.uint8), data_off=np.concatenate(([0], np.cumsum(lens))),
        chunk_size=np.array(cs, np.int64), kind=np.array(kinds), expected=np.concatenate(exp).astype(np.uint32),
        expected_off=np.array(exp_off, np.int64), num_sequences=np.array(nseq, np.int64),
        syn_seed=np.array([s["seed"] for s in syn], np.int64), syn_size=np.array([s["size"] for s in syn], np.int64),
        syn_sha256=np.array([s["sha256"] for s in syn]), syn_chunk_size=np.array([s["chunk_size"] for s in syn]),
        syn_num_sequences=np.array([s["num_sequences"] for s in syn], np.int64),
        syn_index=np.concatenate([s["index"] for s in syn]).astype(np.uint32),
        syn_index_off=np.concatenate(([0], np.cumsum([len(s["index"]) for s in syn]))).astype(np.int64))
    with open(os.path.join(HERE, "fasta_slices.json"), "w") as f:
        json.dump(fasta_slices(), f)
    with open(os.path.join(HERE, "csv_slices.json"), "w") as f:
        json.dump(csv_slices(), f)
    with open(os.path.join(HERE, "vcf_slices.json"), "w") as f:
        json.dump(vcf_slices(), f)
    with open(os.path.join(HERE, "fastq_batches.json"), "w") as f:
        json.dump(fastq_batches(), f)
    print("golden fixtures written:", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    import logging
    logging.disable(logging.CRITICAL)
    main()
