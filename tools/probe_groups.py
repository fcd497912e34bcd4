"""Probe (GPU): FASTA scan time and exactness by index dtype and object offset of the buffer.

    python tools/probe_groups.py [--size BYTES]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd import synth  # noqa: E402
from dataplug_amd.scan import ScanContext  # noqa: E402
from oracle import dpref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1 << 30)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--bases", default=f"{0},{3 << 30},{4 << 30},{8 << 30},{12 << 30}")
    args = ap.parse_args()
    n = args.size
    obj = synth.TiledFasta(16 << 30, seed=1)
    ctx = ScanContext(0)
    d = ctx.workspace("in", n + (64 << 10) + 64)
    out = ctx.workspace("out", 16 * (n // 256 + 1024))
    for base in [int(x) for x in args.bases.split(",")]:
        host = obj.bytes_range(base, base + n + (64 << 10))
        ctx.h2d(d.ptr, host)
        plan = [(base + i * (n // 4), base + (i + 1) * (n // 4)) for i in range(4)]
        rel = [(a - base, b - base) for a, b in plan]
        exp = dpref.fasta_pairs(host, rel) + np.uint64(base)
        chunks = np.ascontiguousarray(np.asarray(plan, np.uint64).reshape(-1))
        for u64 in (False, True):
            if not u64 and base + n + (64 << 10) > (1 << 32):
                continue
            cap = n // 256 + 1024
            res = {"base": base, "u64": u64}
            ctx.timing(True)
            ctx.timing_read()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                ctx.fasta_index_async(d.ptr, len(host), base, 16 << 30, chunks, out.ptr, u64, cap)
                try:
                    cnt, pending, _ = ctx.fasta_result(4)
                except Exception as e:  # report and go on
                    res["error"] = str(e)
                    cnt, pending = 0, np.zeros(4)
            wall = (time.perf_counter() - t0) / args.reps
            ms, k = ctx.timing_read()
            ctx.timing(False)
            got = ctx.d2h(np.empty((cnt, 2), np.uint64 if u64 else np.uint32), out.ptr)
            res.update(kernel_us=round(ms / max(1, k) * 1e3, 1), wall_us=round(wall * 1e6, 1), pairs=int(cnt),
                       exp_pairs=len(exp), pending=pending.tolist(),
                       exact=bool(cnt == len(exp) and np.array_equal(got.astype(np.uint64), exp)))
            if not res["exact"] and cnt:
                bad = np.flatnonzero((got.astype(np.uint64) != exp[:cnt]).any(axis=1)) if cnt <= len(exp) else []
                res["first_bad"] = int(bad[0]) if len(bad) else None
                if len(bad):
                    res["bad_got"] = got[bad[0]].tolist()
                    res["bad_exp"] = exp[bad[0]].tolist()
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
