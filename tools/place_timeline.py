"""Section times of one fasta_place_kernel launch (diagnostics build: tools/build_variants.py diag=DP_DIAG), next to
the map kernel's wave end times, in microseconds from the map kernel's first wave start.

    DPSCAN_LIB=dataplug_amd/lib/libdpscan_v_diag.so python tools/place_timeline.py [--size BYTES]

Per placement block: 0 start (after its ticket), 1 range summaries loaded + wave scans, 2 block scan done,
3 block prefix resolved (look-back), 7 the block's output run known (two barriers later), 4 events staged,
5 output written, 6 dense rescans done.
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
    ap.add_argument("--form", type=int, default=0, help="DP_FORM_FASTA: 0 map + placement kernels, 2 fused")
    args = ap.parse_args()
    n = args.size
    ctx = ScanContext(0)
    ctx.set_form(fasta=args.form)
    host = synth.tiled_fasta_host(n, seed=1)
    d = ctx.workspace("in", n + 64)
    ctx.h2d(d.ptr, host)
    cs = math.ceil(n / 4)
    chunks = np.asarray([(i * cs, min(n, (i + 1) * cs)) for i in range(n // cs)], np.uint64).reshape(-1)
    out = ctx.workspace("out", n // 64)
    for _ in range(3):
        ctx.fasta_index_async(d.ptr, n, 0, n, chunks, out.ptr, False, n // 256)
        ctx.fasta_result(len(chunks) // 2)
    ctx.stream_read(d.ptr, n)                   # the read-only calibration kernel over the same bytes
    ctx.sync()
    ctx.timing(True)
    ctx.timing_read()
    ctx.stream_read(d.ptr, n)
    ctx.sync()
    stream_ms, _ = ctx.timing_read()
    ctx.fasta_index_async(d.ptr, n, 0, n, chunks, out.ptr, False, n // 256)   # the launch the stamps describe
    ctx.fasta_result(len(chunks) // 2)
    span_ms, _ = ctx.timing_read()
    ctx.timing(False)
    words = 1024 * 16 * 8
    buf = np.zeros(words, np.uint64)
    sl, wv = ctypes.c_int(), ctypes.c_int()
    check(_lib.load().dp_debug_profile(ctx.handle, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), words,
                                       ctypes.byref(sl), ctypes.byref(wv)))
    w = buf.reshape(1024, 16, 8).astype(np.int64)
    mp = w[:256]
    live = mp[:, :, 1] > 0
    t0 = mp[:, :, 0][live].min()
    map_end = (mp[:, :, 1][live].max() - t0) / 100.0
    nb = -(-(n // (16 << 10)) // 1024)
    pl = w[512:512 + min(nb, 512), 0, :8]
    us = (pl - t0) / 100.0
    q = lambda a: [round(float(x), 1) for x in np.percentile(a, [0, 50, 100])]
    st = (mp[:, :, 0][live] - t0) / 100.0
    en = (mp[:, :, 1][live] - t0) / 100.0
    res = {"span_us": round(span_ms * 1e3, 1), "stream_us": round(stream_ms * 1e3, 1),
           "map_last_wave_end": round(map_end, 1), "blocks": int(len(pl)),
           "map_wave_start_q0_50_90_100": [round(float(x), 1) for x in np.percentile(st, [0, 50, 90, 100])],
           "map_wave_end_q0_10_50_100": [round(float(x), 1) for x in np.percentile(en, [0, 10, 50, 100])]}
    if len(pl) == 0 or (pl[:, 0] == 0).all():
        print(json.dumps(res), flush=True)
        return
    names = ["start", "loaded", "scanned", "prefix", "staged", "written", "end", "run_bounds"]
    for i, nm in enumerate(names):
        res[nm] = q(us[:, i])
    res["prefix_minus_scanned_med"] = round(float(np.median(us[:, 3] - us[:, 2])), 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
