"""Host-only rate of the parallel gzip inflater (libdpgz dpgz_par_*) vs zlib on one core, on a synthetic FASTQ
member: feed in 4 MiB reads, drain into a 64 MiB buffer (as scan/gzindex.py does), no GPU.

    python tools/gz_par_rate.py [--reads N] [--threads 1,4,8,16] [--region-kib 1024]
"""
from __future__ import annotations

import argparse
import gzip
import json
import os
import sys
import time
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd import gz, synth  # noqa: E402


def run(blob: bytes, threads: int, region: int, out: np.ndarray):
    pi = gz.ParInflate(1 << 22, threads, region_bytes=region)
    t0 = time.perf_counter()
    total = 0
    step = 4 << 20
    mv = memoryview(blob)
    for i in range(0, len(blob), step):
        pi.feed(mv[i:i + step], i + step >= len(blob))
        while True:
            n = pi.read_into(out, 0, len(out))
            if not n:
                break
            total += n
    dt = time.perf_counter() - t0
    st = pi.stats()
    pi.close()
    return total, dt, st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--threads", default="1,4,8,16")
    ap.add_argument("--region-kib", type=int, default=1024)
    args = ap.parse_args()
    raw = synth.fastq(args.reads, seed=5).tobytes()
    blob = gzip.compress(raw, 6)
    t0 = time.perf_counter()
    ref = zlib.decompress(blob, 31)
    tz = time.perf_counter() - t0
    print(json.dumps({"inflated_bytes": len(raw), "gzip_bytes": len(blob),
                      "zlib_1core_GiB_per_s": round(len(raw) / tz / 2**30, 3)}), flush=True)
    out = np.zeros(64 << 20, np.uint8)
    # BGZF: every member inflated independently (gz.bgzf_scan + gz.inflate_members), whole object at once
    bg = np.frombuffer(synth.bgzf(raw, level=6), np.uint8)
    a, ln, ol, used = gz.bgzf_scan(bg)
    oo = np.concatenate(([0], np.cumsum(ol)[:-1])).astype(np.uint64)
    big = np.zeros(int(ol.sum()), np.uint8)
    for th in (int(x) for x in args.threads.split(",")):
        t0 = time.perf_counter()
        gz.inflate_members(bg, a, ln, oo, ol, big.ctypes.data, th)
        dt = time.perf_counter() - t0
        print(json.dumps({"bgzf_threads": th, "members": len(a), "GiB_per_s": round(len(big) / dt / 2**30, 3),
                          "ok": big.tobytes() == ref}), flush=True)
    for th in (int(x) for x in args.threads.split(",")):
        n, dt, st = run(blob, th, args.region_kib << 10, out)
        print(json.dumps({"threads": th, "GiB_per_s": round(n / dt / 2**30, 3), "ok": n == len(ref),
                          "batches": st["batches"], "rejected": st["rejected"], "wall_ms": round(dt * 1e3, 1),
                          **{k: round(v / 1e6, 1) for k, v in st.items() if k.startswith("ns_")}}), flush=True)


if __name__ == "__main__":
    main()
