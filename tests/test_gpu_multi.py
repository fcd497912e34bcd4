"""Multi-GPU product path on the GPU box (one MI355X: device lists like [0]*8 rehearse the split).

* The reference's canonical plan (chunk_size = ceil(size / 4), examples/fasta_example.py:23) fills 8 groups:
  chunks are cut at byte boundaries (scan.objects.fasta_pieces) and stitched; the index equals the C oracle's
  for the whole chunks, with cuts inside header lines and on the cs == num_chunks - 1 plan.
* Persistent per-GPU workers: a second co.preprocess of a same-size object allocates nothing
  (dp_alloc_counts).
* One scan stream per device: eight contexts launching scans concurrently on device 0 each see launch times
  within 2x of a solo launch.
* The per-chunk joblib route on the loky process backend (docs/preprocessing.md:6-15 of the reference): the
  CloudObject is pickled into spawned workers that initialise HIP and scan their chunks over loopback S3."""
import math
import threading

import numpy as np
import pytest

from dataplug_amd import synth
from dataplug_amd.cloudobject import CloudObject
from dataplug_amd.storage import LoopbackS3Server, MemoryStore

pytestmark = pytest.mark.gpu


def _mem(name):
    MemoryStore._named.pop(name, None)
    return {"endpoint_url": f"memory://{name}"}


def _co(fmt, data: bytes, key: str, cfg):
    co = CloudObject.from_s3(fmt, f"s3://data/{key}", fetch=False, s3_config=cfg)
    try:
        co.storage.head_bucket(Bucket="data")
    except Exception:
        co.storage.create_bucket(Bucket="data")
    co.storage.put_object(Body=data, Bucket="data", Key=key)
    return CloudObject.from_s3(fmt, f"s3://data/{key}", s3_config=cfg)


def _index(co, dt=np.uint32):
    return np.frombuffer(co.storage.get_object(Bucket=co.meta_path.bucket, Key=co.meta_path.key)["Body"].read(), dt)


def _long_headers(n, seed):
    """Records whose header lines run 0-200 KB (so byte cuts land inside header lines), '>' inside sequence
    lines and runs of '>'."""
    rng = np.random.default_rng(seed)
    parts, total = [], 0
    while total < n:
        h = b">" * int(rng.integers(1, 3)) + b"h" * int(rng.choice([5, 3000, 200_000])) + b"\n"
        body = np.frombuffer(b"ACGT>", np.uint8)[rng.integers(0, 5, int(rng.integers(0, 50_000)))]
        w = int(rng.integers(1, 200))
        parts.append(h + b"".join(body[i:i + w].tobytes() + b"\n" for i in range(0, len(body), w)))
        total += len(parts[-1])
    return np.frombuffer(b"".join(parts)[:n], np.uint8).copy()


@pytest.mark.parametrize("kind", ["synth", "long_headers"])
@pytest.mark.parametrize("groups", [8, 5, 3])
def test_canonical_plan_cut_over_groups(kind, groups):
    from oracle import cpu_ref, dpref
    from dataplug_amd.formats.genomics.fasta import FASTA
    from dataplug_amd.scan.objects import fasta_split
    n = (24 << 20) + 4321
    a = synth.fasta(n, 90 + groups) if kind == "synth" else _long_headers(n, 90 + groups)
    cs = math.ceil(n / 4)
    plan = cpu_ref.chunk_plan(n, cs)
    pieces, _, gs = fasta_split(plan, groups, n)
    assert len(gs) == groups
    assert any(not p.first for p in pieces) == (groups % len(plan) != 0)     # 3 chunks (floor plan): 3 whole
    co = _co(FASTA, a.tobytes(), f"canon_{kind}_{groups}", _mem(f"canon_{kind}_{groups}"))
    co.preprocess(chunk_size=cs, parallel_config={"dataplug_devices": [0] * groups})
    exp = dpref.fasta_pairs(a, plan)
    assert np.array_equal(_index(co), exp.reshape(-1).astype(np.uint32))


def test_quirk_plan_cut_over_eight_groups():
    """chunk_size == num_chunks - 1 (every map job reads to EOF, handler.py:36-38) split over 8 groups."""
    from oracle import cpu_ref, dpref
    from dataplug_amd.formats.genomics.fasta import FASTA
    cs = 300
    a = _long_headers(cs * (cs + 1) + 7, 5)
    a[::997] = 10
    assert len(a) // cs == cs + 1
    co = _co(FASTA, a.tobytes(), "quirk8", _mem("quirk8"))
    co.preprocess(chunk_size=cs, parallel_config={"dataplug_devices": [0] * 8})
    exp = dpref.fasta_pairs(a, cpu_ref.chunk_plan(len(a), cs))
    assert np.array_equal(_index(co), exp.reshape(-1).astype(np.uint32))


def test_second_preprocess_allocates_nothing():
    """dataplug_devices=[0, 0]: each group runs on its device's persistent worker, whose context keeps its
    pinned staging and HBM workspace; the second same-size object adds no device or pinned allocation."""
    from dataplug_amd.formats.genomics.fasta import FASTA
    from dataplug_amd.scan._lib import alloc_counts
    from oracle import cpu_ref, dpref
    n = (32 << 20) + 999
    cs = math.ceil(n / 4)
    counts = []
    for i in range(3):
        a = synth.fasta(n, 200 + i)
        co = _co(FASTA, a.tobytes(), f"warm{i}", _mem(f"warm{i}"))
        co.preprocess(chunk_size=cs, parallel_config={"dataplug_devices": [0, 0]})
        assert np.array_equal(_index(co), dpref.fasta_pairs(a, cpu_ref.chunk_plan(n, cs)).reshape(-1).astype(np.uint32))
        counts.append(alloc_counts())
    print("alloc counts after each preprocess (device, pinned host):", counts)
    assert counts[1] == counts[2] and counts[0] == counts[1], counts


def test_eight_contexts_share_the_scan_stream():
    """Eight contexts on device 0, each with its own stream, launching scans from eight threads at once: the
    scans run one after another on the device's scan stream, and every context's average scan (HIP events
    around the kernels) stays within 2x of a solo scan of the same bytes."""
    from oracle import cpu_ref
    from dataplug_amd.scan import ScanContext
    n = 256 << 20
    a = synth.tiled_fasta_host(n, seed=3)
    plan = np.asarray(cpu_ref.chunk_plan(n, n // 4), np.uint64).reshape(-1)

    def setup():
        c = ScanContext(0)
        d = c.workspace("in", n + 64)
        c.h2d(d.ptr, a)
        o = c.workspace("out", n // 64)
        return c, d, o

    def run(c, d, o, reps):
        c.timing(True)
        c.timing_read()
        for _ in range(reps):
            c.fasta_index_async(d.ptr, n, 0, n, plan, o.ptr, False, n // 512)
            c.fasta_result(len(plan) // 2)
        ms, k = c.timing_read()
        return ms / max(1, k)

    solo_ctx = setup()
    run(*solo_ctx, 3)
    solo = run(*solo_ctx, 10)
    ctxs = [setup() for _ in range(8)]
    res = [None] * 8

    def worker(i):
        res[i] = run(*ctxs[i], 10)

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    print(f"solo scan {solo * 1e3:.1f} us; 8 contexts: " + ", ".join(f"{r * 1e3:.1f}" for r in res) + " us")
    assert all(r < 2 * solo for r in res), (solo, res)
    for c in [solo_ctx] + ctxs:
        c[0].close()


def test_loky_process_backend_over_loopback():
    """parallel_config={"backend": "loky", "n_jobs": 2}: the reference's per-chunk joblib route on spawned
    worker processes (the CloudObject and its storage client pickled into them, picklableS3.py:132-162),
    each initialising HIP and scanning its chunks on GPU 0; the stored index equals the oracle's."""
    from oracle import cpu_ref, dpref
    from dataplug_amd.formats.genomics.fasta import FASTA
    n = (6 << 20) + 77
    a = synth.fasta(n, 17)
    cs = math.ceil(n / 5)
    with LoopbackS3Server() as srv:
        co = _co(FASTA, a.tobytes(), "loky.fasta", srv.storage_config)
        co.preprocess(chunk_size=cs, parallel_config={"backend": "loky", "n_jobs": 2})
        exp = dpref.fasta_pairs(a, cpu_ref.chunk_plan(n, cs))
        assert np.array_equal(_index(co), exp.reshape(-1).astype(np.uint32))
        assert co.attributes.num_sequences == len(exp)
