"""DELIM kernel variants over the same resident bytes (HIP events, GB/s of input): FASTQ / CSV / VCF
shapes, every '\\n' (uint64 / u16b) vs every 4th + 1 (the FASTQ read ends) vs a byte that never occurs
(no events: the scan's read + count floor).

    python tools/probe_delim_modes.py [--gib 8] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=8)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    size = int(args.gib * (1 << 30))
    ctx = ScanContext(0)
    d = ctx.workspace("in", size + 64)
    out = ctx.workspace("out", size // 4 + (1 << 20))
    gens = {"fastq": lambda: synth.fastq(200_000, seed=3), "csv": lambda: synth.csv(64 * (1 << 20) - 333, 9),
            "vcf": lambda: synth.vcf(64 * (1 << 20) - 333, 9)}
    for name, gen in gens.items():
        base = gen()
        host = synth.tiled_host(base, size)
        nl = int(np.count_nonzero(host == 10))
        ctx.h2d(d.ptr, host)
        del host
        res = {"shape": name, "bytes": size, "newlines": nl}
        cases = {"none": (0x07, 1, 0, True), "all_u64": (10, 1, 0, True), "k4_u64": (10, 4, 1, True)}
        for c, (delim, k, add, u64) in cases.items():
            cap = size // 4 // 8

            def run():
                ctx.delim_index_async(d.ptr, size, 0, 0, size, delim, k, add, out.ptr, u64, cap)
                ctx.delim_result()

            t = kernel_time(ctx, run, args.reps)
            res[f"{c}_GBps"] = round(size / t / 1e9, 1)
        rg = np.array([0, size], np.uint64)

        def run_u16b():
            ctx.delim_ranges_async(d.ptr, size, 0, rg, 10, 1, 0, 0, out.ptr, 3, nl + 64)
            ctx.delim_ranges_result(1)

        t = kernel_time(ctx, run_u16b, args.reps)
        res["all_u16b_GBps"] = round(size / t / 1e9, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
