"""Same-process A/B of FASTA forms: one resident configs[1]-shaped object, one context per form (dp_ctx_set_form), the
same chunk plan, launches alternated rep by rep (HIP events on the scan stream), every launch's pairs compared with
the first form's and, once, with the C oracle.  Same buffers for every form (DESIGN.md §5's placement effect alike).

    python tools/fasta_form_ab.py [--forms 0,2] [--sizes-gib 4,0.5] [--reps 10] [--chunks 4]
    python tools/fasta_form_ab.py --lib-b dataplug_amd/lib/libdpscan_v_X.so   # form0: the shipped library, form1: X
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd import synth  # noqa: E402
from dataplug_amd.scan import ScanContext  # noqa: E402
from oracle import cpu_ref, dpref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--forms", default="0,2")
    ap.add_argument("--sizes-gib", default="4,0.5")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("--lib-b", default=None, help="A/B of two builds (default form each): form0 = the shipped "
                    "library, form1 = this one")
    args = ap.parse_args()
    ctxs = {}
    if args.lib_b:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from lib_ab import context_on
        forms = [0, 1]
        ctxs = {0: ScanContext(0), 1: context_on(args.lib_b)}
    else:
        forms = [int(x) for x in args.forms.split(",")]
        for f in forms:
            c = ScanContext(0)
            c.set_form(fasta=f)
            ctxs[f] = c
    c0 = ctxs[forms[0]]
    for size in (int(float(x) * (1 << 30)) for x in args.sizes_gib.split(",")):
        host = synth.tiled_fasta_host(size, seed=1)
        d = c0.workspace("in", size + 64)
        c0.h2d(d.ptr, host)
        plan = cpu_ref.chunk_plan(size, math.ceil(size / args.chunks))
        ch = np.ascontiguousarray(np.asarray(plan, np.uint64).reshape(-1))
        cap = size // 256 + 1024
        outs = {f: c.workspace("out", 4 * 2 * cap) for f, c in ctxs.items()}

        def run(f):
            ctxs[f].fasta_index_async(d.ptr, size, 0, size, ch, outs[f].ptr, False, cap)
            return ctxs[f].fasta_result(len(plan))[0]
        n = {f: run(f) for f in forms}
        for c in ctxs.values():
            c.timing(True)
            c.timing_read()
        t = {f: [] for f in forms}
        for rep in range(args.reps):
            order = forms[rep % len(forms):] + forms[:rep % len(forms)]
            for f in order:
                run(f)
                t[f].append(round(ctxs[f].timing_read()[0] * 1e3, 1))
        for c in ctxs.values():
            c.timing(False)
        got = {f: ctxs[f].d2h(np.empty(2 * n[f], np.uint32), outs[f].ptr) for f in forms}
        equal = all(n[f] == n[forms[0]] and np.array_equal(got[f], got[forms[0]]) for f in forms)
        oracle_ok = None
        if not args.no_oracle:
            oracle_ok = bool(np.array_equal(got[forms[0]].astype(np.uint64),
                                            dpref.fasta_pairs(host, plan).reshape(-1)))
        line = {"size_gib": size / (1 << 30), "pairs": int(n[forms[0]]), "equal": bool(equal), "oracle": oracle_ok}
        for f in forms:
            line[f"form{f}_us"] = float(np.median(t[f]))
            line[f"form{f}_all"] = t[f]
        base = line[f"form{forms[0]}_us"]
        for f in forms[1:]:
            line[f"form{f}_over_form{forms[0]}"] = round(line[f"form{f}_us"] / base, 4)
        print(json.dumps(line), flush=True)
        del host
        if not equal or oracle_ok is False:
            sys.exit(1)


if __name__ == "__main__":
    main()
