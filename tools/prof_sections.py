"""In-kernel section breakdown of scan_kernel (needs lib/libdpscan_prof.so: python -m dataplug_amd.build --prof).

    DPSCAN_LIB=dataplug_amd/lib/libdpscan_prof.so python tools/prof_sections.py [--size BYTES]

Data waves:   0 wait for the input buffer (vmcnt)  1 phase A  2 publish / ready polls before a blocking wait
              3 blocking wait for the coordinator's prefix  4 phase B  5 ready polls + prefetch issue  6 drain
              7 the tail's waits for the last prefixes.
Coordinator:  0 compose + publish AGG  1 look-back attempts  2 resolve + hand-off  3 idle (nothing to do).
Reported as the mean over workgroups of each slot's share of the wave's total time.
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

DATA = ["wait_buf", "phase_a", "pre_wait", "wait_ready", "phase_b", "post_prefetch", "drain", "tail_wait"]
COORD = ["compose", "lookback_try", "resolve", "idle", "-", "-", "-", "-"]


def read(ctx, grid):
    n = 1024 * 16 * 8
    buf = np.zeros(n, np.uint64)
    sl, wv = ctypes.c_int(), ctypes.c_int()
    check(_lib.load().dp_debug_profile(ctx.handle, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n,
                                       ctypes.byref(sl), ctypes.byref(wv)))
    return buf.reshape(1024, 16, 8)[:grid].astype(np.float64)


def summarize(p):
    data = p[:, :15, :]
    coord = p[:, 15, :]
    dtot = data.sum(-1, keepdims=True)
    coord = coord.copy()
    spins = coord[:, 4].copy()
    failed = coord[:, 5].copy()
    resolved = coord[:, 6].copy()
    coord[:, 4:7] = 0
    ctot = coord.sum(-1, keepdims=True)
    out = {"data_ticks_per_wave": float(dtot.mean())}
    out.update({f"data_{n}": round(float((data / dtot)[..., i].mean()), 3) for i, n in enumerate(DATA) if n != "-"})
    out.update({f"coord_{n}": round(float((coord / ctot)[..., i].mean()), 3) for i, n in enumerate(COORD) if n != "-"})
    out["coord_attempts_per_wg"] = round(float(spins.mean()), 1)
    out["coord_incomplete_per_wg"] = round(float(failed.mean()), 1)
    out["coord_resolved_per_wg"] = round(float(resolved.mean()), 1)
    busy = data[..., 1] + data[..., 4] + data[..., 5]          # phase A + phase B + post, per (wg, wave)
    out["busy_by_wave"] = [round(float(x), 3) for x in (busy / dtot[..., 0]).mean(0)]
    out["wait_ready_by_wave"] = [round(float(x), 3) for x in (data[..., 3] / dtot[..., 0]).mean(0)]
    tot_wg = dtot[..., 0].mean(1)
    out["wg_time_spread"] = [round(float(np.percentile(tot_wg, q) / tot_wg.mean()), 3) for q in (0, 50, 100)]
    out["busy_wg_spread"] = [round(float(np.percentile(busy.sum(1), q) / busy.sum(1).mean()), 3) for q in (0, 50, 100)]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4 << 30)
    args = ap.parse_args()
    size = args.size
    ctx = ScanContext(0)
    grid, _ = ctx.geometry()
    host = synth.tiled_fasta_host(size, seed=1)
    d = ctx.workspace("in", size + 64)
    ctx.h2d(d.ptr, host)
    out = ctx.workspace("out", size // 4)
    cs = math.ceil(size / 4)
    chunks = np.asarray([(i * cs, min(size, (i + 1) * cs)) for i in range(size // cs)], np.uint64).reshape(-1)
    res = {}

    def run(name, fn):
        fn()
        ctx.sync()
        ctx.timing(True)
        ctx.timing_read()
        fn()
        ms, _ = ctx.timing_read()
        ctx.timing(False)
        r = summarize(read(ctx, grid))
        r["kernel_ms"] = round(ms, 4)
        r["GBps"] = round(size / ms / 1e6, 1)
        res[name] = r
        print(name, json.dumps(r), flush=True)

    run("fasta_synth", lambda: (ctx.fasta_index_async(d.ptr, size, 0, size, chunks, out.ptr, False, size // 256),
                                ctx.fasta_result(len(chunks) // 2)))
    run("delim_on_fasta", lambda: (ctx.delim_index_async(d.ptr, size, 0, 0, size, 10, 1, 0, out.ptr, False, size // 16),
                                   ctx.delim_result()))
    run("delim_rare", lambda: (ctx.delim_index_async(d.ptr, size, 0, 0, size, ord("#"), 1, 0, out.ptr, False, size // 16),
                               ctx.delim_result()))
    csv = synth.tiled_host(synth.csv(64 * (1 << 20) - 333, 9), size)
    nl = int(np.count_nonzero(csv == 10))
    ctx.h2d(d.ptr, csv)
    del csv
    out_nl = ctx.workspace("out_nl", 8 * nl + 1024)
    run("csv_newline_u64", lambda: (ctx.delim_index_async(d.ptr, size, 0, 0, size, 10, 1, 0, out_nl.ptr, True, nl + 64),
                                    ctx.delim_result()))
    line = np.frombuffer(b"ACGT" * 15 + b"\n", np.uint8)
    ctx.h2d(d.ptr, np.resize(line, size))
    run("fasta_no_gt", lambda: (ctx.fasta_index_async(d.ptr, size, 0, size, chunks, out.ptr, False, size // 256),
                                ctx.fasta_result(len(chunks) // 2)))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
