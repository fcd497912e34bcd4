"""Per-wave start/end times of one fasta_map_kernel launch (diagnostics build: tools/build_variants.py diag=DP_DIAG).

    DPSCAN_LIB=dataplug_amd/lib/libdpscan_v_diag.so python tools/map_timeline.py [--size BYTES]

Prints, in microseconds from the launch's first wave start: the spread of wave starts, the distribution of
wave and workgroup end times, per-XCC medians of workgroup end times, and the ranges per wave.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4 << 30)
    args = ap.parse_args()
    n = args.size
    ctx = ScanContext(0)
    host = synth.tiled_fasta_host(n, seed=1)
    d = ctx.workspace("in", n + 64)
    ctx.h2d(d.ptr, host)
    cs = math.ceil(n / 4)
    chunks = np.asarray([(i * cs, min(n, (i + 1) * cs)) for i in range(n // cs)], np.uint64).reshape(-1)
    out = ctx.workspace("out", n // 64)
    for _ in range(3):
        ctx.fasta_index_async(d.ptr, n, 0, n, chunks, out.ptr, False, n // 256)
        ctx.fasta_result(len(chunks) // 2)
    words = 1024 * 16 * 8
    buf = np.zeros(words, np.uint64)
    sl, wv = ctypes.c_int(), ctypes.c_int()
    check(_lib.load().dp_debug_profile(ctx.handle, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), words,
                                       ctypes.byref(sl), ctypes.byref(wv)))
    w = buf.reshape(1024, 16, 8)[:256].astype(np.int64)
    live = w[:, :, 1] > 0
    t0 = w[:, :, 0][live].min()
    start = (w[:, :, 0] - t0) / 100.0
    end = (w[:, :, 1] - t0) / 100.0
    wg_end = np.where(live, end, -1).max(axis=1)
    xcc = w[:, 0, 3]
    q = lambda a: [round(float(x), 1) for x in np.percentile(a, [0, 10, 50, 90, 100])]
    res = {"wave_start_pct": q(start[live]), "wave_end_pct": q(end[live]), "wg_end_pct": q(wg_end),
           "ranges_per_wave": q(w[:, :, 2][live]),
           "wg_end_median_by_xcc": {int(x): round(float(np.median(wg_end[xcc == x])), 1) for x in np.unique(xcc)},
           "wg_end_median_by_blockidx_mod8": {k: round(float(np.median(wg_end[k::8])), 1) for k in range(8)},
           "intra_wg_end_spread_median": round(float(np.median(np.where(live, end, np.nan).max(1) -
                                                                np.where(live, end, np.nan).min(1))), 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
