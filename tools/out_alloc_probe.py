"""Does the newline kernel's time depend on where its output buffer lives?  One resident VCF / CSV object, one
context, several separately allocated output buffers (optionally after fragmenting the device heap with large
allocations freed again); every rep runs the same launch into each buffer in turn (HIP events on the scan stream).

    python tools/out_alloc_probe.py [--content vcf] [--size-gib 4] [--buffers 6] [--reps 8] [--fragment-gib 0]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--content", default="vcf")
    ap.add_argument("--size-gib", type=float, default=4)
    ap.add_argument("--buffers", type=int, default=6)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--mode", type=int, default=4)
    ap.add_argument("--fragment-gib", type=float, default=0, help="allocate and free this much in 1.5 GiB pieces first")
    ap.add_argument("--contexts", type=int, default=1, help="spread the buffers over this many scan contexts (each "
                    "with its own chunk table and look-back descriptors)")
    args = ap.parse_args()
    size = int(args.size_gib * (1 << 30))
    ctx = ScanContext(0)
    if args.fragment_gib:
        n = int(args.fragment_gib / 1.5)
        for i in range(n):
            ctx.workspace(f"frag{i}", int(1.5 * (1 << 30)))
        for i in range(0, n, 2):                # every other piece back: holes between live ones
            ctx._bufs.pop(f"frag{i}").free()
    obj = (synth.tiled_csv if args.content == "csv" else synth.tiled_vcf)(size, seed=1)
    d = ctx.workspace("in", size + 64)
    step = 2 << 30
    stage = np.empty(min(step, size), np.uint8)
    for p in range(0, size, step):
        ctx.h2d(d.ptr + p, obj.bytes_range(p, min(size, p + step), out=stage))
    del stage
    n_exp = obj.count_range(0, size)
    cap = n_exp + 1024
    rg = np.asarray([0, size], np.uint64)
    ob = ScanContext.out_bytes(cap, args.mode, rg)
    ctxs = [ctx] + [ScanContext(0) for _ in range(args.contexts - 1)]
    cx = [ctxs[k % len(ctxs)] for k in range(args.buffers)]
    outs = [c.workspace(f"out{k}", ob) for k, c in enumerate(cx)]
    times = [[] for _ in outs]
    st = []

    def run(c, o):
        c.delim_ranges_async(d.ptr, size, 0, rg, 10, 1, 0, 0, o.ptr, args.mode, cap)
        return c.delim_ranges_result(1)[0]
    for c, o in zip(cx, outs):
        assert run(c, o) == n_exp
    for c in ctxs:
        c.timing(True)
        c.timing_read()
    for rep in range(args.reps):
        ctx.stream_read(d.ptr, size)
        ctx.sync()
        ms, _ = ctx.timing_read()
        st.append(round(ms * 1e3, 1))
        for k, (c, o) in enumerate(zip(cx, outs)):
            run(c, o)
            ms, _ = c.timing_read()
            times[k].append(round(ms * 1e3, 1))
    for c in ctxs:
        c.timing(False)
    res = {"content": args.content, "size_gib": args.size_gib, "mode": args.mode, "fragment_gib": args.fragment_gib,
           "stream_median_us": float(np.median(st)),
           "buffers": [{"ctx": k % len(ctxs), "addr_mod_2m": o.ptr % (2 << 20), "addr_gib": round(o.ptr / (1 << 30), 3),
                        "median_us": float(np.median(t)), "all_us": t} for k, (o, t) in enumerate(zip(outs, times))]}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
