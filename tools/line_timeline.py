"""Per-step phase times of line_kernel (diagnostics build: tools/build_variants.py diag=DP_DIAG).

    DPSCAN_LIB=dataplug_amd/lib/libdpscan_v_diag.so python tools/line_timeline.py [--content sparse|csv|vcf] [--gib 2]

Each of waves 0, 1, 8 and 15 of the first 256 workgroups stamps the realtime clock (100 MHz) at 8 points of
every step (dpscan.hip LTL): 0 after the step barrier, 1 after b[0]'s wait, 2 after wave 0's AGG publication
(and its window reduction in DP_LINE_LATE=0), 3 after rows(0) + b[0]'s reload, 4 after b[1]'s wait (+ the window
reduction in DP_LINE_LATE=1), 5 after rows(1) + the range record, 6 after the step's placements, 7 after the slot
stall + b[1]'s reload + the window loads.  Prints the median / mean of each phase per wave over the steady
steps, the step period, how often a step stalled, and the launch's tail.
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
from dataplug_amd.scan import ScanContext, _lib  # noqa: E402
from dataplug_amd.scan._lib import check  # noqa: E402

BASE = 1024 * 16 * 8
STEPS, WAVES = 64, 4
PHASES = ["wait_b0", "w0_block", "rows0_reload", "wait_b1", "rows1_rec", "place", "stall_reload_win", "barrier"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--content", default="sparse", choices=["sparse", "csv", "vcf"])
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--mode", type=int, default=4, choices=[3, 4], help="csv/vcf out_mode: 4 u8s (stored), 3 u16b")
    args = ap.parse_args()
    n = int(args.gib * (1 << 30))
    ctx = ScanContext(0)
    if args.content == "sparse":                              # the size sweep's '>' index, uint64 offsets
        host = synth.tiled_fasta_host(n, seed=1)
    else:                                                     # the stored '\n' index (out_mode 4 or 3)
        host = (synth.tiled_csv if args.content == "csv" else synth.tiled_vcf)(n, seed=1).bytes_range(0, n)
    d = ctx.workspace("in", n + 64)
    ctx.h2d(d.ptr, host)
    del host
    cap = n // 16
    ranges = np.asarray([0, n], np.uint64)
    out = ctx.workspace("out", max(n // 2, ScanContext.out_bytes(cap, args.mode, ranges)))
    for _ in range(3):
        if args.content == "sparse":
            ctx.delim_index_async(d.ptr, n, 0, 0, n, 62, 1, 0, out.ptr, True, n // 256)
            ctx.delim_result()
        else:
            ctx.delim_ranges_async(d.ptr, n, 0, ranges, 10, 1, 0, 0, out.ptr, args.mode, cap)
            ctx.delim_ranges_result(1)
    words = BASE + 256 * STEPS * WAVES * 8
    buf = np.zeros(words, np.uint64)
    sl, wv = ctypes.c_int(), ctypes.c_int()
    check(_lib.load().dp_debug_profile(ctx.handle, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), words,
                                       ctypes.byref(sl), ctypes.byref(wv)))
    t = buf[BASE:].reshape(256, STEPS, WAVES, 8).astype(np.int64)
    t0 = t[:, 0, 0, 0][t[:, 0, 0, 0] > 0]
    t0 = t0[t0 >= t0.max() - 5000]                          # the last launch's step-0 stamps (50 us of spread)
    start = int(t0.min())                                    # its start: anything older is a stale stamp
    valid = t >= start
    t = np.where(valid, t - start, -1)
    # a step is complete when all 8 stamps of wave 0 are valid; the steady steps skip the first and last two
    nsteps = (t[:, :, 0, 7] >= 0).sum(axis=1)
    res = {"content": args.content, "gib": args.gib, "steps_per_wg": [int(x) for x in np.percentile(nsteps, [0, 50, 100])]}
    per = {}
    for w, name in enumerate(["w0", "w1", "w8", "w15"]):
        ph = {k: [] for k in PHASES}
        for b in range(256):
            for k in range(2, max(2, nsteps[b] - 2)):
                s = t[b, k, w]
                nxt = t[b, k + 1, w, 0]
                if (s < 0).any() or nxt < 0:
                    continue
                dd = list(np.diff(s)) + [nxt - s[7]]
                for name_, v in zip(PHASES, dd):
                    ph[name_].append(v / 100.0)
        per[name] = {k: (round(float(np.median(v)), 2), round(float(np.mean(v)), 2)) for k, v in ph.items() if v}
    res["phase_us_median_mean"] = per
    period = []
    stalls = 0
    tot = 0
    for b in range(256):
        for k in range(2, max(2, nsteps[b] - 2)):
            a, c = t[b, k, 0, 0], t[b, k + 1, 0, 0]
            if a >= 0 and c >= 0:
                period.append((c - a) / 100.0)
            s6, s7 = t[b, k, 0, 6], t[b, k, 0, 7]
            if s6 >= 0 and s7 >= 0:
                tot += 1
                stalls += (s7 - s6) > 100          # > 1 us in the stall + reload + window phase
    res["step_period_us_pct"] = [round(float(x), 2) for x in np.percentile(period, [10, 50, 90])]
    res["stall_steps_frac"] = round(stalls / max(1, tot), 3)
    tail_start = [t[b, nsteps[b], 0, 0] for b in range(256) if nsteps[b] < STEPS and t[b, nsteps[b], 0, 0] >= 0]
    tail_end = [t[b, nsteps[b], 0, 1] for b in range(256) if nsteps[b] < STEPS and t[b, nsteps[b], 0, 1] >= 0]
    if tail_start and tail_end:
        res["tail_us"] = {"loop_end_pct": [round(float(x) / 100, 1) for x in np.percentile(tail_start, [0, 50, 100])],
                          "kernel_end_pct": [round(float(x) / 100, 1) for x in np.percentile(tail_end, [0, 50, 100])]}
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
