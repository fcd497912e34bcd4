"""Where does a CSV co.preprocess() spend its time end to end (memory store)?  A configs[2]-shaped CSV object in the
in-process memory store, one warm call, then a cProfile of the next (top functions by cumulative time).

    python tools/e2e_profile.py [--gib 4] [--kind csv|fasta] [--top 30] [--http]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import math
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4)
    ap.add_argument("--kind", default="csv")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--http", action="store_true", help="through the loopback S3 server (a child process)")
    args = ap.parse_args()
    from dataplug_amd import synth
    from dataplug_amd.cloudobject import CloudObject
    from dataplug_amd.formats.generic.csv import CSV
    from dataplug_amd.formats.genomics.fasta import FASTA
    from dataplug_amd.storage import MemoryStore
    size = int(args.gib * (1 << 30))
    store = MemoryStore.named("e2e_prof")
    bucket = "data"
    for b in (bucket, bucket + ".meta"):
        store.create_bucket(b)
    if args.kind == "csv":
        host = synth.tiled_csv(size, seed=9).bytes_range(0, size)
        fmt, call_kw = CSV, {}
    else:
        host = synth.tiled_fasta_host(size, seed=1)
        fmt, call_kw = FASTA, {"chunk_size": math.ceil(size / 4)}
    store.put(bucket, "x", host)
    del host
    cfg = {"endpoint_url": "memory://e2e_prof"}
    srv = None
    if args.http:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from e2e_legs import _Server
        srv = _Server(19073, [(f"{bucket}/x", args.kind, size, 9 if args.kind == "csv" else 1)], [bucket + ".meta"])
        srv.wait_ready()
        cfg = {"endpoint_url": srv.url}
    co = CloudObject.from_s3(fmt, f"s3://{bucket}/x", s3_config=cfg)
    for i in range(3):
        t = time.perf_counter()
        co.preprocess(force=True, **call_kw)
        print(f"call {i}: {time.perf_counter() - t:.4f} s", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    t = time.perf_counter()
    co.preprocess(force=True, **call_kw)
    dt = time.perf_counter() - t
    pr.disable()
    print(f"profiled call: {dt:.4f} s ({size / dt / (1 << 30):.2f} GiB/s)", flush=True)
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(args.top)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(args.top)
    print(s.getvalue())
    if srv is not None:
        srv.stop()


if __name__ == "__main__":
    main()
