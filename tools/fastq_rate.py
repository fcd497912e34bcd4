"""FASTQ.gz per-read index rates (BASELINE configs[4], fastqgz_example.py shape), for DESIGN.md §6.

    python tools/fastq_rate.py [--reads N] [--reps R]

A synthetic FASTQ (100 bp reads, gzip level 6) in an in-process store (memory://):
* `co.preprocess()` of FASTQGZip end to end: GET, host inflate with access points (libdpgz), H2D, the
  newline scan on the GPU, D2H, window table + read index PUTs;
* its stages: the inflate alone, and the host-bytes -> GPU newline index -> host round trip;
* the device-resident read-end index of the inflated stream (dp_delim_index every_k = 4, emit_add = 1),
  timed with HIP events, checked against the reads' own line ends.
"""
from __future__ import annotations

import argparse
import gzip
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd import gz as gzidx  # noqa: E402
from dataplug_amd import synth  # noqa: E402
from dataplug_amd.cloudobject import CloudObject  # noqa: E402
from dataplug_amd.formats.genomics.fastq import FASTQGZip, load_read_index  # noqa: E402
from dataplug_amd.scan import get_context  # noqa: E402
from dataplug_amd.scan import objects as so  # noqa: E402
from dataplug_amd.storage import MemoryStore  # noqa: E402

GiB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    t0 = time.perf_counter()
    raw = synth.fastq(args.reads, seed=5)
    blob = gzip.compress(raw.tobytes(), 6)
    res = {"reads": args.reads, "inflated_bytes": int(len(raw)), "gzip_bytes": len(blob),
           "gen_s": round(time.perf_counter() - t0, 1)}
    print(json.dumps(res), flush=True)
    store = MemoryStore.named("fq")
    store.create_bucket("genomics")
    store.create_bucket("genomics.meta")
    store.put("genomics", "r.fastq.gz", blob)
    co = CloudObject.from_s3(FASTQGZip, "s3://genomics/r.fastq.gz", s3_config={"endpoint_url": "memory://fq"})
    co.preprocess(force=True)                               # warm: pandas/pyarrow, context, buffers
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        co.preprocess(force=True)
        ts.append(time.perf_counter() - t0)
    nl = np.flatnonzero(raw == 10).astype(np.uint64)
    exp_ends = nl[3::4] + np.uint64(1)
    assert np.array_equal(load_read_index(co), exp_ends)
    t = min(ts)
    res.update({"preprocess_s": round(t, 3), "preprocess_inflated_GiB_per_s": round(len(raw) / t / GiB, 3),
                "preprocess_gzip_GiB_per_s": round(len(blob) / t / GiB, 3)})
    # stages
    t0 = time.perf_counter()
    inflated, _ = gzidx.build_index(blob, span=1 << 20)
    t_inf = time.perf_counter() - t0
    assert np.array_equal(np.asarray(inflated), raw)
    so.record_index_bytes(inflated)
    t0 = time.perf_counter()
    got, n_nl = so.record_index_bytes(inflated)
    t_rt = time.perf_counter() - t0
    assert n_nl == len(nl)
    res.update({"stage_inflate_GiB_per_s": round(len(raw) / t_inf / GiB, 3),
                "stage_host_to_gpu_index_to_host_GiB_per_s": round(len(raw) / t_rt / GiB, 2)})
    # device-resident read-end index (every 4th newline + 1), HIP events around each launch
    ctx = get_context(0)
    n = len(raw)
    d = ctx.workspace("fq_in", n + 64)
    ctx.h2d(d.ptr, raw)
    cap = len(exp_ends) + 1024
    out = ctx.workspace("fq_out", 8 * cap)
    ctx.delim_index_async(d.ptr, n, 0, 0, n, 10, 4, 1, out.ptr, True, cap)
    ctx.delim_result()
    ctx.timing(True)
    ctx.timing_read()
    for _ in range(10):
        ctx.delim_index_async(d.ptr, n, 0, 0, n, 10, 4, 1, out.ptr, True, cap)
        n_out, _ = ctx.delim_result()
    ms, launches = ctx.timing_read()
    ctx.timing(False)
    ends = ctx.d2h(np.empty(n_out, np.uint64), out.ptr)
    assert np.array_equal(ends, exp_ends)
    k = ms / 1e3 / launches
    res.update({"device_read_index_kernel_us": round(k * 1e6, 1),
                "device_read_index_GiB_per_s": round(n / k / GiB, 1),
                "device_read_index_alg_GBps": round((n + 8.0 * n_out) / k / 1e9, 1),
                "device_read_index_frac_of_8TBps": round((n + 8.0 * n_out) / k / 8e12, 3),
                "verified": True})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
