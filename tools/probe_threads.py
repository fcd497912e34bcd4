"""Probe (GPU): several host threads scanning their own chunk groups of one object on ONE device.

    python tools/probe_threads.py [--workers 4] [--size BYTES per worker] [--reps 4] [--serial-upload]

Per worker and rep: kernel time (HIP events), pair count and exactness vs the oracle, and whether the
input bytes on the device still equal the host bytes afterwards (d2h compare).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd import synth  # noqa: E402
from dataplug_amd.scan import ScanContext  # noqa: E402
from dataplug_amd.scan.objects import fasta_groups  # noqa: E402
from oracle import dpref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--size", type=int, default=4 << 30)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--serial-upload", action="store_true")
    ap.add_argument("--one-ctx", action="store_true", help="one context per worker (default two, alternating)")
    args = ap.parse_args()
    W = args.workers
    size = args.size * W
    cs = size // (4 * W)
    plan = [(i * cs, (i + 1) * cs) for i in range(4 * W)]
    groups = fasta_groups(plan, W, size)
    obj = synth.TiledFasta(size, seed=1)
    u64 = size > (1 << 32)
    bar = threading.Barrier(W)
    up_lock = threading.Lock()
    out = [None] * W

    def work(k):
        g = groups[k]
        ctxs = [ScanContext(0)] if args.one_ctx else [ScanContext(0), ScanContext(0)]
        host = obj.bytes_range(g.lo, g.buf_hi)
        d = ctxs[0].workspace("in", len(host) + 64)
        if args.serial_upload:
            with up_lock:
                ctxs[0].h2d(d.ptr, host)
        else:
            ctxs[0].h2d(d.ptr, host)
        rel = [(a - g.lo, b - g.lo) for a, b in g.chunks(plan)]
        exp = dpref.fasta_pairs(host, rel) + np.uint64(g.lo)
        chunks = g.chunks(plan)
        recs = []
        bar.wait()
        for r in range(args.reps):
            c = ctxs[r % len(ctxs)]
            c.timing(True)
            c.timing_read()
            try:
                pairs, pending, _ = c.fasta_index(d.ptr, len(host), g.lo, size, chunks, u64=u64)
                ok = bool((pending == -1).all() and np.array_equal(pairs.astype(np.uint64), exp))
                n = len(pairs)
                err = None
            except Exception as e:
                ok, n, err = False, -1, str(e)
            ms, kn = c.timing_read()
            c.timing(False)
            recs.append({"rep": r, "us": round(ms / max(1, kn) * 1e3, 1), "n": n, "ok": ok, "err": err})
        back = ctxs[0].d2h(np.empty(len(host), np.uint8), d.ptr)
        out[k] = {"worker": k, "lo": g.lo, "bytes": len(host), "exp": len(exp),
                  "input_intact": bool(np.array_equal(back, host)), "reps": recs}
        for c in ctxs:
            c.close()

    th = [threading.Thread(target=work, args=(k,)) for k in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
