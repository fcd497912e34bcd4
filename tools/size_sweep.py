"""Fixed vs per-byte cost of the scan kernels: kernel time (HIP events) over object sizes, next to the
read-only stream kernel over the same bytes.  A linear fit t = a + b * size separates the launch's fixed
start/tail cost (a) from its steady-state rate (1 / b).

    python tools/size_sweep.py [--sizes-gib 1,2,4,8,16] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd import synth  # noqa: E402
from dataplug_amd.scan import ScanContext  # noqa: E402


def kernel_time(ctx, fn, reps):
    fn()
    ctx.sync()
    ctx.timing(True)
    ctx.timing_read()
    for _ in range(reps):
        fn()
    ctx.sync()
    ms, n = ctx.timing_read()
    ctx.timing(False)
    return ms / max(1, n) / 1e3


def fit(xs, ts):
    b, a = np.polyfit(np.asarray(xs, float), np.asarray(ts, float), 1)
    return a, b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-gib", default="1,2,4,8,16")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    sizes = [int(float(x) * (1 << 30)) for x in args.sizes_gib.split(",")]
    top = max(sizes)
    ctx = ScanContext(0)
    d = ctx.workspace("in", top + 64)
    ctx.h2d(d.ptr, synth.tiled_fasta_host(top, seed=1))
    out = ctx.workspace("out", top // 32)
    rows = {"stream": [], "fasta": [], "newline": []}
    for size in sizes:
        cs = math.ceil(size / 4)
        chunks = np.asarray([(i * cs, min(size, (i + 1) * cs)) for i in range(size // cs)], np.uint64).reshape(-1)
        u64 = size > (1 << 32)

        def fasta():
            ctx.fasta_index_async(d.ptr, size, 0, size, chunks, out.ptr, u64, top // 256)
            ctx.fasta_result(len(chunks) // 2)

        def newline():
            ctx.delim_index_async(d.ptr, size, 0, 0, size, 62, 1, 0, out.ptr, True, top // 256)
            ctx.delim_result()

        t = {"stream": kernel_time(ctx, lambda: ctx.stream_read(d.ptr, size), args.reps),
             "fasta": kernel_time(ctx, fasta, args.reps),
             "newline": kernel_time(ctx, newline, args.reps)}
        for k, v in t.items():
            rows[k].append(v)
        print(json.dumps({"size_gib": size / (1 << 30), **{f"{k}_us": round(v * 1e6, 1) for k, v in t.items()},
                          **{f"{k}_GBps": round(size / v / 1e9, 1) for k, v in t.items()}}), flush=True)
    for k, ts in rows.items():
        a, b = fit(sizes, ts)
        print(json.dumps({"kernel": k, "fixed_us": round(a * 1e6, 1), "steady_GBps": round(1 / b / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
