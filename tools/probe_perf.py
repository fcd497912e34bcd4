"""Perf probe (GPU): calibration stream read vs the scan kernels on different inputs, one process.

    python tools/probe_perf.py [--size BYTES] [--reps N]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd import synth  # noqa: E402
from dataplug_amd.scan import ScanContext  # noqa: E402


def timed(ctx, fn, reps):
    fn()
    ctx.sync()
    ctx.timing(True)
    ctx.timing_read()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    ctx.sync()
    wall = (time.perf_counter() - t0) / reps
    ms, n = ctx.timing_read()
    ctx.timing(False)
    return ms / max(1, n) / 1e3, wall


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4 << 30)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-stream", action="store_true", help="skip the stream-read calibration")
    ap.add_argument("--only", choices=["fasta", "delim", "nogt", "csv", "vcf"],
                    help="run one workload (for rocprofv3 --pmc)")
    args = ap.parse_args()
    size = args.size
    ctx = ScanContext(0)
    host = synth.tiled_fasta_host(size, seed=1)
    d = ctx.workspace("in", size + 64)
    ctx.h2d(d.ptr, host)
    res = {"lib": os.path.basename(os.environ.get("DPSCAN_LIB", "libdpscan.so"))}
    for bpc in (() if args.no_stream else (1, 2, 4, 8, 16)):
        k, w = timed(ctx, lambda: ctx.stream_read(d.ptr, size, bpc), args.reps)
        res[f"stream_read_bpc{bpc}_GBps"] = round(size / k / 1e9, 1)
        print(bpc, res, flush=True)
    cs = math.ceil(size / 4)
    chunks = np.asarray([(i * cs, min(size, (i + 1) * cs)) for i in range(size // cs)], np.uint64).reshape(-1)
    out = ctx.workspace("out", size // 4)
    cap = size // 256

    def fasta():
        ctx.fasta_index_async(d.ptr, size, 0, size, chunks, out.ptr, False, cap)
        ctx.fasta_result(len(chunks) // 2)

    if args.only in (None, "fasta"):
        k, w = timed(ctx, fasta, args.reps)
        res["fasta_synth_kernel_GBps"] = round(size / k / 1e9, 1)
        res["fasta_synth_wall_GBps"] = round(size / w / 1e9, 1)

    def delim():
        ctx.delim_index_async(d.ptr, size, 0, 0, size, 10, 1, 0, out.ptr, False, size // 16)
        ctx.delim_result()

    if args.only in (None, "delim"):
        k, w = timed(ctx, delim, args.reps)
        res["delim_on_fasta_kernel_GBps"] = round(size / k / 1e9, 1)

    # FASTA-shaped bytes without any '>': the row fast path everywhere
    line = np.frombuffer(b"ACGT" * 15 + b"\n", np.uint8)
    plain = np.resize(line, size)
    if args.only in (None, "nogt"):
        ctx.h2d(d.ptr, plain)
        k, w = timed(ctx, fasta, args.reps)
        res["fasta_no_gt_kernel_GBps"] = round(size / k / 1e9, 1)
    # BASELINE configs[2] / [3] shapes (cities.csv rows, sample.vcf rows): the newline index (uint64) of
    # [0, size); algorithmic bytes = N + 8 * L
    for name, gen in (("csv", synth.csv), ("vcf", synth.vcf)):
        if args.only not in (None, name):
            continue
        data = synth.tiled_host(gen(64 * (1 << 20) - 333, 9), size)
        nl = int(np.count_nonzero(data == 10))
        ctx.h2d(d.ptr, data)
        del data
        out_nl = ctx.workspace("out_nl", 8 * nl + 1024)

        def newline(cap=nl + 64):
            ctx.delim_index_async(d.ptr, size, 0, 0, size, 10, 1, 0, out_nl.ptr, True, cap)
            ctx.delim_result()

        k, w = timed(ctx, newline, args.reps)
        res[f"{name}_newline_kernel_GBps"] = round(size / k / 1e9, 1)
        res[f"{name}_newline_alg_GBps"] = round((size + 8.0 * nl) / k / 1e9, 1)
        res[f"{name}_newlines"] = nl
    g, ub = ctx.geometry()
    res["grid"] = g
    res["unit_bytes"] = ub
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
