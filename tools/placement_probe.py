"""Probe the placement of N separately allocated device buffers in one process (ScanContext.placement_ratio: the
read-while-writing / read-only time ratio of the calibration kernels), all held at once, and time line_kernel's u8s
newline index over a CSV-shaped object in each, to check that the ratio predicts the scan's slow placement mode.

    python tools/placement_probe.py [--gib 4] [--n 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd import synth  # noqa: E402
from dataplug_amd.scan import ScanContext  # noqa: E402
from dataplug_amd.scan.device import DeviceBuffer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    n = int(args.gib * (1 << 30))
    ctx = ScanContext(0)
    host = synth.tiled_csv(n, seed=9).bytes_range(0, n)
    bufs = [DeviceBuffer(ctx, n + 64) for _ in range(args.n)]
    for i, b in enumerate(bufs):
        ratio = ctx.placement_ratio(b, n)
        ctx.h2d(b.ptr, host)
        ctx.sync()
        rg = [(0, n)]
        ctx.delim_ranges(b.ptr, n, 0, rg, out_mode=4)          # warm: sizes the outputs
        ctx.sync()
        ctx.timing(True)
        ctx.timing_read()
        for _ in range(args.reps):
            ctx.delim_ranges(b.ptr, n, 0, rg, out_mode=4)
        ms, k = ctx.timing_read()
        ctx.timing(False)
        print(json.dumps({"buffer": i, "ratio": round(ratio, 4), "scan_us": round(ms / max(1, k) * 1e3, 1)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
