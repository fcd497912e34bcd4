"""Does the newline kernel's time depend on the input buffer it reads?  The same 4 GiB of a synthetic VCF / CSV
object uploaded into several separately allocated device buffers of different sizes (the launch reads the first
``--size-gib`` of each); every rep runs the stream kernel and the newline launch (u8s) over each buffer in turn, on
one context with one output buffer (HIP events on the scan stream).

    python tools/in_alloc_probe.py [--content vcf] [--size-gib 4] [--buffers-gib 4,8,16,4] [--reps 4]
"""
from __future__ import annotations

import argparse
import ctypes
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
    ap.add_argument("--buffers-gib", default="4,8,16,4")
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--mode", type=int, default=4)
    ap.add_argument("--cap0", action="store_true", help="output capacity 0: counts and tables only, no entries")
    ap.add_argument("--alloc", default="", help="comma list per buffer: d (library hipMalloc) | c (hipExtMallocWithFlags "
                    "contiguous) | u (uncached) | f (fine-grained); default all d")
    ap.add_argument("--out-alloc", default="d", help="d | c | u: the output and stream_rw buffers' allocation")
    ap.add_argument("--lib-b", default=None, help="a second libdpscan build: its stream_rw timed beside (same buffers)")
    ap.add_argument("--wpr", type=float, default=0.025, help="stream_rw's write bytes per read byte (0: reads only, "
                    "in the same lockstep group pattern)")
    args = ap.parse_args()
    size = int(args.size_gib * (1 << 30))
    ctx = ScanContext(0)
    obj = (synth.tiled_csv if args.content == "csv" else synth.tiled_vcf)(size, seed=1)
    host = obj.bytes_range(0, size)
    bufs = []
    kinds = args.alloc.split(",") if args.alloc else []
    hip = None

    class Raw:                                        # a buffer from hipExtMallocWithFlags (flags: HIP's hipDeviceMalloc*)
        def __init__(self, nbytes, flags):
            p = ctypes.c_void_p()
            rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(flags))
            if rc != 0:
                raise RuntimeError(f"hipExtMallocWithFlags({nbytes}, {flags}) = {rc}")
            self.ptr, self.nbytes = p.value, nbytes
    for k, g in enumerate(float(x) for x in args.buffers_gib.split(",")):
        kind = kinds[k] if k < len(kinds) else "d"
        nbytes = max(size + 64, int(g * (1 << 30)))
        if kind == "d":
            b = ctx.workspace(f"in{k}", nbytes)
        else:
            if hip is None:
                hip = ctypes.CDLL("libamdhip64.so")
            b = Raw(nbytes, {"c": 4, "u": 3, "f": 1}[kind])
        b.kind = kind
        ctx.h2d(b.ptr, host)
        bufs.append(b)
    del host
    n_exp = obj.count_range(0, size)
    cap = 0 if args.cap0 else n_exp + 1024
    rg = np.asarray([0, size], np.uint64)
    def alloc(name, nbytes, kind):
        nonlocal hip
        if kind == "d":
            return ctx.workspace(name, nbytes)
        if hip is None:
            hip = ctypes.CDLL("libamdhip64.so")
        return Raw(nbytes, {"c": 4, "u": 3, "f": 1}[kind])
    out = alloc("out", ScanContext.out_bytes(cap, args.mode, rg), args.out_alloc)

    def run(b):
        ctx.delim_ranges_async(b.ptr, size, 0, rg, 10, 1, 0, 0, out.ptr, args.mode, cap)
        try:
            return ctx.delim_ranges_result(1)[0]
        except Exception as e:                      # (--cap0) the capacity error carries the count
            return getattr(e, "needed", None)
    for b in bufs:
        assert run(b) == n_exp
    ctx.timing(True)
    ctx.timing_read()
    st = [[] for _ in bufs]
    rw = [[] for _ in bufs]
    rwb = [[] for _ in bufs]
    nlb = [[] for _ in bufs]
    ctx_b = None
    if args.lib_b:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from lib_ab import context_on
        ctx_b = context_on(args.lib_b)
        out_b = ctx_b.workspace("out", ScanContext.out_bytes(max(cap, 1), args.mode, rg))

        def run_b(b):
            ctx_b.delim_ranges_async(b.ptr, size, 0, rg, 10, 1, 0, 0, out_b.ptr, args.mode, cap)
            return ctx_b.delim_ranges_result(1)[0]
        for b in bufs:
            run_b(b)                                  # (a timing-probe build may write no index)
        ctx_b.timing(True)
        ctx_b.timing_read()
    nl = [[] for _ in bufs]
    wpr = args.wpr                                    # 0.025: the u8s index's write bytes per read byte on VCF
    mix = alloc("mix", int(wpr * size) + (1 << 20), args.out_alloc)
    for _ in range(args.reps):
        for k, b in enumerate(bufs):
            ctx.stream_read(b.ptr, size)
            ctx.sync()
            st[k].append(round(ctx.timing_read()[0] * 1e3, 1))
            ctx.stream_rw(b.ptr, size, mix.ptr, wpr)
            ctx.sync()
            rw[k].append(round(ctx.timing_read()[0] * 1e3, 1))
            if ctx_b is not None:
                ctx_b.stream_rw(b.ptr, size, mix.ptr, wpr)
                ctx_b.sync()
                rwb[k].append(round(ctx_b.timing_read()[0] * 1e3, 1))
            run(b)
            nl[k].append(round(ctx.timing_read()[0] * 1e3, 1))
            if ctx_b is not None:
                run_b(b)
                nlb[k].append(round(ctx_b.timing_read()[0] * 1e3, 1))
    ctx.timing(False)
    print(json.dumps({"content": args.content, "size_gib": args.size_gib, "mode": args.mode, "cap0": args.cap0,
                      "buffers": [{"gib": round(b.nbytes / (1 << 30), 2), "kind": b.kind, "addr_gib": round(b.ptr / (1 << 30), 2),
                                   "stream_us": float(np.median(s)), "stream_rw_us": float(np.median(w)),
                                   "stream_rw_b_us": float(np.median(wb)) if wb else None,
                                   "newline_b_us": float(np.median(tb)) if tb else None,
                                   "newline_us": float(np.median(t)), "newline_all": t}
                                  for b, s, w, wb, t, tb in zip(bufs, st, rw, rwb, nl, nlb)]}), flush=True)


if __name__ == "__main__":
    main()
