"""Same-process A/B of two libdpscan builds on the newline index: both libraries loaded side by side (ctypes keeps their
symbols apart), one context each, the same resident input and the same output form, launches alternated rep by rep,
outputs compared byte for byte.  Same buffers for both, so the placement effect of DESIGN.md §5 touches both alike.

    python tools/lib_ab.py --b dataplug_amd/lib/libdpscan_v_X.so [--a dataplug_amd/lib/libdpscan.so]
                           [--content csv,vcf] [--sizes-gib 4,16] [--reps 8] [--out-mode 4]
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


def context_on(path: str) -> ScanContext:
    """A ScanContext whose calls go to the library at `path` (guard-checked like the loader does)."""
    if os.path.abspath(path) == os.path.abspath(_lib.LIB_PATH):
        return ScanContext(0)
    _lib.guard_check(path)
    lib = ctypes.CDLL(path)
    for name, res, args in _lib.SIGNATURES:
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    c = object.__new__(ScanContext)
    c.lib = lib
    h = ctypes.c_void_p()
    _lib.check(lib.dp_ctx_create(0, ctypes.byref(h)))
    c.handle, c.device, c._bufs, c._pinned, c._get_pool = h, 0, {}, {}, None
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", default=_lib.LIB_PATH)
    ap.add_argument("--b", required=True)
    ap.add_argument("--content", default="csv,vcf")
    ap.add_argument("--sizes-gib", default="4,16")
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--out-mode", type=int, default=4)
    ap.add_argument("--no-compare", action="store_true", help="a timing probe whose index differs (reported, not fatal)")
    args = ap.parse_args()
    ctxs = {"a": context_on(args.a), "b": context_on(args.b)}
    sizes = [int(float(x) * (1 << 30)) for x in args.sizes_gib.split(",")]
    top = max(sizes)
    mode = args.out_mode
    d = ctxs["a"].workspace("in", top + 64)
    for content in args.content.split(","):
        obj = (synth.tiled_csv if content == "csv" else synth.tiled_vcf)(top, seed=1)
        step = 2 << 30
        stage = np.empty(min(step, top), np.uint8)
        for p in range(0, top, step):
            ctxs["a"].h2d(d.ptr + p, obj.bytes_range(p, min(top, p + step), out=stage))
        del stage
        cap_top = obj.count_range(0, top) + 1024
        outs = {k: c.workspace("out", ScanContext.out_bytes(cap_top, mode, np.asarray([0, top], np.uint64)))
                for k, c in ctxs.items()}
        for size in sizes:
            n_exp = obj.count_range(0, size)
            cap = n_exp + 1024
            rg = np.asarray([0, size], np.uint64)
            t = {"a": [], "b": []}

            def run(k):
                ctxs[k].delim_ranges_async(d.ptr, top, 0, rg, 10, 1, 0, 0, outs[k].ptr, mode, cap)
                return ctxs[k].delim_ranges_result(1)[0]
            for k in ctxs:
                assert run(k) == n_exp
                ctxs[k].timing(True)
                ctxs[k].timing_read()
            for rep in range(args.reps):
                for k in (("a", "b") if rep % 2 == 0 else ("b", "a")):
                    run(k)
                    t[k].append(round(ctxs[k].timing_read()[0] * 1e3, 1))
            for c in ctxs.values():
                c.timing(False)
            res = {}
            for k, c in ctxs.items():
                dt = np.uint8 if mode == 4 else np.uint16
                res[k] = [c.d2h(np.empty(n_exp, dt), outs[k].ptr), c.block_table(outs[k].ptr, cap, rg, mode)]
                if mode == 4:
                    res[k].append(c.sub_table(outs[k].ptr, cap, rg))
            equal = all(np.array_equal(x, y) for x, y in zip(res["a"], res["b"]))
            ma, mb = float(np.median(t["a"])), float(np.median(t["b"]))
            print(json.dumps({"content": content, "size_gib": size / (1 << 30), "out_mode": mode, "a_us": ma, "b_us": mb,
                              "b_over_a": round(mb / ma, 4), "equal": equal, "a_all": t["a"], "b_all": t["b"]}),
                  flush=True)
            if not equal and not args.no_compare:
                sys.exit(1)


if __name__ == "__main__":
    main()
