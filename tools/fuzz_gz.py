"""Time-bounded randomized campaign for the parallel gzip inflater (libdpgz dpgz_par_*, host only): random
streams against zlib's streaming index (gz.InflateStream), as tests/test_gzpar_cpu.py does for fixed cases.

    python tools/fuzz_gz.py [--seconds 180] [--seed 1] [--out gpurun_out/fuzz_gz.json]

Streams: FASTQ, CSV, random bytes, runs, and mixes of them; 1-4 members with zero padding between some;
levels 0-9, strategies default / filtered / Huffman-only / RLE / fixed; sync and full flushes at random
points.  Engine settings: 1-8 threads, regions of 4 KiB-2 MiB, feeds of 1 B-8 MiB, span 16 KiB-1 MiB.  The
inflated bytes, every access point (offsets, bits, member starts, preceding byte) and every window must equal
zlib's.  Exits non-zero on the first mismatch (the stream is kept in gpurun_out/fuzz_gz_fail.npz).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

from dataplug_amd import synth  # noqa: E402
from test_gzpar_cpu import _par, _zlib_ref  # noqa: E402

STRATEGIES = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED]


def payload(rng, size):
    kind = int(rng.integers(0, 5))
    if kind == 0:
        return synth.fastq(max(1, size // 240), int(rng.integers(0, 1 << 30))).tobytes()[:size]
    if kind == 1:
        return synth.csv(max(64, size), int(rng.integers(0, 1 << 30))).tobytes()[:size]
    if kind == 2:
        return rng.integers(0, 256, size, dtype=np.uint8).tobytes()
    if kind == 3:
        return bytes(rng.choice([0, 65, 10], size=size).astype(np.uint8))
    parts = [payload(rng, size // 3) for _ in range(3)]
    return b"".join(parts)


def member(rng, data):
    level = int(rng.integers(0, 10))
    strat = STRATEGIES[int(rng.integers(0, len(STRATEGIES)))]
    c = zlib.compressobj(level, zlib.DEFLATED, 31, 8, strat)
    out = []
    i = 0
    while i < len(data):
        j = min(len(data), i + int(rng.integers(1, max(2, len(data) // 3 + 2))))
        out.append(c.compress(data[i:j]))
        if j < len(data) and rng.random() < 0.3:
            out.append(c.flush(zlib.Z_SYNC_FLUSH if rng.random() < 0.7 else zlib.Z_FULL_FLUSH))
        i = j
    out.append(c.flush())
    return b"".join(out)


def stream(rng):
    size = int(np.exp(rng.uniform(np.log(1), np.log(24 << 20))))
    n = int(rng.integers(1, 5))
    blob = b""
    for k in range(n):
        blob += member(rng, payload(rng, max(0, size // n)))
        if k + 1 < n and rng.random() < 0.3:
            blob += b"\0" * int(rng.integers(1, 64))
    return blob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="gpurun_out/fuzz_gz.json")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    rng = np.random.default_rng(args.seed)
    stats = {"streams": 0, "inflated_bytes": 0, "points": 0, "batches": 0, "rejected": 0}
    t0 = last = time.time()
    while time.time() - t0 < args.seconds:
        blob = stream(rng)
        span = int(rng.choice([16 << 10, 256 << 10, 1 << 20]))
        threads = int(rng.integers(1, 9))
        region = int(rng.choice([4 << 10, 64 << 10, 256 << 10, 1 << 20, 2 << 20]))
        if len(blob) < (64 << 10):
            step = int(rng.choice([1, 4096, 1 << 20]))
        else:
            step = int(rng.choice([1 << 14, 1 << 20, 8 << 20]))
        exp, epts, ewin = _zlib_ref(blob, span)
        got, gpts, gwin, st = _par(blob, span, threads, region, step)
        ok = got == exp and len(gpts) == len(epts) and gwin == ewin
        if ok:
            for f in ("in_byte", "out_byte", "bits", "member_start"):
                ok = ok and np.array_equal(gpts[f], epts[f])
        if not ok:
            np.savez_compressed("gpurun_out/fuzz_gz_fail.npz", blob=np.frombuffer(blob, np.uint8), span=span,
                                threads=threads, region=region, step=step)
            print(json.dumps({"FAIL": True, "len": len(blob), "span": span, "threads": threads, "region": region,
                              "step": step}), flush=True)
            sys.exit(1)
        stats["streams"] += 1
        stats["inflated_bytes"] += len(exp)
        stats["points"] += len(epts)
        stats["batches"] += st["batches"]
        stats["rejected"] += st["rejected"]
        if time.time() - last > 20:
            last = time.time()
            print(json.dumps({"t": round(last - t0), **stats}), flush=True)
    stats.update({"seconds": round(time.time() - t0, 1), "seed": args.seed, "ok": True})
    with open(args.out, "w") as f:
        json.dump(stats, f)
    print(json.dumps(stats), flush=True)


if __name__ == "__main__":
    main()
