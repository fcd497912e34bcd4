"""Per-unit timeline of one scan_kernel<FASTA> launch (profiling build: python tools/build_variants.py prof=DP_PROF).

    DPSCAN_LIB=dataplug_amd/lib/libdpscan_v_prof.so python tools/timeline.py [--size BYTES] [--out file.npz]

For every workgroup b (< 256) and its k-th step (the unit it claimed for it), the kernel stamps the realtime clock (100 MHz)
when (0) the unit's AGG descriptor is published, (1) the coordinator resolved its prefix, (2) data wave 0
finished phase A of it (DP_TL_CLAIM builds: the coordinator claimed it); word 3 holds the step's unit index (dynamic assignment).  This prints, per round k, medians over
workgroups, in microseconds from the launch's first stamp, plus the derived look-back latency: the time
from the moment unit u's whole window was published (max AGG time over units u-G+1 .. u-1 and u's own
previous prefix) to u's resolution.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd import synth  # noqa: E402
from dataplug_amd.scan import ScanContext, _lib  # noqa: E402
from dataplug_amd.scan._lib import check  # noqa: E402

TL_BASE, TL_UNITS = 256 * 16 * 8, 96


def read_timeline(ctx):
    n = 1024 * 16 * 8
    buf = np.zeros(n, np.uint64)
    sl, wv = ctypes.c_int(), ctypes.c_int()
    check(_lib.load().dp_debug_profile(ctx.handle, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n,
                                       ctypes.byref(sl), ctypes.byref(wv)))
    return buf[TL_BASE:TL_BASE + 256 * TL_UNITS * 4].reshape(256, TL_UNITS, 4).astype(np.int64)


def analyse(tl, grid, nunits):
    t = tl[:, :, :3]
    t0 = t[t > 0].min()
    us = np.where(t > 0, (t - t0) / 100.0, np.nan)              # 100 MHz ticks -> us
    K = (nunits + grid - 1) // grid
    # unit index -> (b, k)
    pub = np.full(nunits, np.nan)
    res = np.full(nunits, np.nan)
    w2 = np.full(nunits, np.nan)
    for b in range(grid):
        for k in range(TL_UNITS):
            if tl[b, k, 1] <= 0:
                continue
            u = int(tl[b, k, 3])
            if u < nunits:
                pub[u], res[u], w2[u] = us[b, k, 0], us[b, k, 1], us[b, k, 2]
    # a unit's window is published once every earlier unit back to one already resolved has its AGG
    # (approximation: the 255 previous units' AGGs and the resolution of the unit 256 back)
    ready = np.full(nunits, np.nan)
    for u in range(1, nunits):
        lo = max(0, u - grid + 1)
        w = np.nanmax(pub[lo:u]) if u > lo else 0.0
        if u >= grid:
            w = max(w, res[u - grid])
        ready[u] = max(w, pub[u])
    lat = res - ready
    rows = []
    for k in range(min(K + 8, TL_UNITS)):
        sel = slice(k * grid, min(nunits, (k + 1) * grid))
        if sel.start >= nunits:
            break
        rows.append({
            "k": k,
            "w2_med": round(float(np.nanmedian(w2[sel])), 1),
            "pub_med": round(float(np.nanmedian(pub[sel])), 1),
            "pub_spread": round(float(np.nanmax(pub[sel]) - np.nanmin(pub[sel])), 1),
            "res_med": round(float(np.nanmedian(res[sel])), 1),
            "lag_res_pub": round(float(np.nanmedian(res[sel] - pub[sel])), 1),
            "lookback_lat": round(float(np.nanmedian(lat[sel])), 1),
        })
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4 << 30)
    ap.add_argument("--out", default=None)
    ap.add_argument("--pre-stream", type=int, default=0,
                    help="bytes of a read-only stream kernel enqueued right before the profiled scan (no host gap)")
    args = ap.parse_args()
    size = args.size
    ctx = ScanContext(0)
    grid, unit = ctx.geometry()
    host = synth.tiled_fasta_host(size, seed=1)
    d = ctx.workspace("in", size + 64)
    ctx.h2d(d.ptr, host)
    out = ctx.workspace("out", size // 4)
    cs = math.ceil(size / 4)
    chunks = np.asarray([(i * cs, min(size, (i + 1) * cs)) for i in range(size // cs)], np.uint64).reshape(-1)
    nunits = sum(-(-(min(size, (i + 1) * cs) - i * cs + (i * cs) % 16) // unit) for i in range(size // cs))
    for _ in range(2):
        if args.pre_stream:
            ctx.stream_read(d.ptr, min(size, args.pre_stream))
        ctx.fasta_index_async(d.ptr, size, 0, size, chunks, out.ptr, False, size // 256)
        ctx.fasta_result(len(chunks) // 2)
    tl = read_timeline(ctx)
    if args.out:
        np.savez_compressed(args.out, tl=tl, grid=grid, nunits=nunits)
    rows = analyse(tl, grid, nunits)
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
