"""Same-box probe of the FASTA index launch on a 4 GiB synthetic object (the configs[1] plan): average span
of the scan kernels (HIP events) over --reps launches, bit-exact check of the last one against the C oracle.

    DPSCAN_LIB=dataplug_amd/lib/libdpscan_v_<name>.so python tools/probe_fasta2.py [--size BYTES] [--reps 20]

Run it under `rocprofv3 --kernel-trace --stats` to split the span per kernel (tools/rocpd_stats.py).
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4 << 30)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-verify", action="store_true")
    args = ap.parse_args()
    n = args.size
    ctx = ScanContext(0)
    host = synth.tiled_fasta_host(n, seed=1)
    d = ctx.workspace("in", n + 64)
    ctx.h2d(d.ptr, host)
    cs = math.ceil(n / 4)
    plan = [(i * cs, min(n, (i + 1) * cs)) for i in range(n // cs)]
    chunks = np.asarray(plan, np.uint64).reshape(-1)
    cap = n // 256 + 1024
    out = ctx.workspace("out", 8 * cap + 16)
    for _ in range(3):
        ctx.fasta_index_async(d.ptr, n, 0, n, chunks, out.ptr, False, cap)
        npairs, _, _ = ctx.fasta_result(len(plan))
    ctx.timing(True)
    ctx.timing_read()
    for _ in range(args.reps):
        ctx.fasta_index_async(d.ptr, n, 0, n, chunks, out.ptr, False, cap)
        npairs, pending, _ = ctx.fasta_result(len(plan))
    ms, k = ctx.timing_read()
    us = ms / k * 1e3
    ok = None
    if not args.no_verify:
        from oracle import dpref
        got = ctx.d2h(np.empty((npairs, 2), np.uint32), out.ptr)
        ok = bool((pending == -1).all() and np.array_equal(got.astype(np.uint64), dpref.fasta_pairs(host, plan)))
    alg = n + 8 * npairs
    print(json.dumps({"lib": os.path.basename(os.environ.get("DPSCAN_LIB", "libdpscan.so")),
                      "size": n, "span_us": round(us, 1),
                      "alg_TBps": round(alg / us / 1e6, 3), "frac": round(alg / us / 1e6 / 8.0, 4), "pairs": npairs,
                      "bit_exact": ok}), flush=True)


if __name__ == "__main__":
    main()
