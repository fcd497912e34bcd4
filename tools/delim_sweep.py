"""Newline index: its kernel forms over launch sizes, on CSV / VCF / FASTA bytes (same box).

Contexts on device 0 pinned to one form each -- the one-pass look-back kernel (DP_DELIM_TWOPASS_MAX=0), the
two-kernel form (map + placement: DP_DELIM_TWOPASS_MAX above every size) and, round 4, the lockstep one-pass
line_kernel (DP_DELIM_FORM=line) -- plus the library's default choice, run `dp_delim_ranges` over [0, size) of
the same resident
object in the stored CSV/VCF form (out_mode 3: uint16 low words + the 64 KiB block table) and time the scan
with HIP events.  Both outputs are compared byte for byte at every size, and the linear fit t = a + b * size
per form gives its fixed cost and steady rate: where the lines cross is the crossover the library's
kDelimTwoPassMax encodes.

    python tools/delim_sweep.py [--content csv,vcf,fasta] [--sizes-gib 0.0625,0.25,0.5,1,2,4] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd import synth  # noqa: E402
from dataplug_amd.scan import ScanContext  # noqa: E402


def make_ctx(twopass_max=None, form=None):
    env = {"DP_DELIM_TWOPASS_MAX": None if twopass_max is None else str(twopass_max), "DP_DELIM_FORM": form}
    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    ctx = ScanContext(0)
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    if twopass_max is not None:
        assert ctx.forms()[1] == twopass_max, ctx.forms()
    return ctx


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--content", default="csv,vcf,fasta")
    ap.add_argument("--sizes-gib", default="0.0625,0.25,0.5,1,2,4")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--forms", default="onepass,twokernel,line,default")
    ap.add_argument("--no-check", action="store_true", help="timing probes with wrong results: keep going")
    args = ap.parse_args()
    sizes = [int(float(x) * (1 << 30)) for x in args.sizes_gib.split(",")]
    top = max(sizes)
    makers = {"onepass": lambda: make_ctx(0, "one"), "twokernel": lambda: make_ctx(1 << 62, "two"),
              "line": lambda: make_ctx(None, "line"), "auto": lambda: make_ctx(None, "auto"),
              "default": lambda: make_ctx()}
    forms = {k: makers[k]() for k in args.forms.split(",")}
    ctx0 = next(iter(forms.values()))
    d = ctx0.workspace("in", top + 64)
    for content in args.content.split(","):
        if content == "fasta":
            host = synth.tiled_fasta_host(top, seed=1)
        else:
            obj = (synth.tiled_csv if content == "csv" else synth.tiled_vcf)(top, seed=1)
            host = obj.bytes_range(0, top)
        ctx0.h2d(d.ptr, host)
        del host
        cap = top // 16
        rows = {k: [] for k in forms}
        for size in sizes:
            ranges = np.asarray([0, size], np.uint64)
            ob = ScanContext.out_bytes(cap, 3, ranges)
            res = {}
            line = {"content": content, "size_gib": size / (1 << 30)}
            for name, ctx in forms.items():
                out = ctx.workspace("out", ob)

                def run():
                    ctx.delim_ranges_async(d.ptr, top, 0, ranges, 10, 1, 0, 0, out.ptr, 3, cap)
                    return ctx.delim_ranges_result(1)

                n = run()[0]
                ctx.timing(True)
                ctx.timing_read()
                for _ in range(args.reps):
                    run()
                ms, k = ctx.timing_read()
                ctx.timing(False)
                t = ms / max(1, k) / 1e3
                rows[name].append(t)
                words = ctx.d2h(np.empty(n, np.uint16), out.ptr)
                res[name] = (n, words, ctx.block_table(out.ptr, cap, ranges))
                line[f"{name}_us"] = round(t * 1e6, 1)
                line[f"{name}_GBps"] = round(size / t / 1e9, 1)
                # roofline fraction on algorithmic bytes: input + 2 B per entry + 8 B per 64 KiB block
                line[f"{name}_frac"] = round((size + 2 * n + 8 * len(res[name][2])) / t / 8e12, 4)
            vals = list(res.values())
            a = vals[0]
            line["entries"] = a[0]
            line["equal"] = bool(all(b[0] == a[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
                                     for b in vals[1:]))
            print(json.dumps(line), flush=True)
            if not line["equal"] and not args.no_check:
                print("MISMATCH", flush=True)
                sys.exit(1)
        for name, ts in rows.items():
            bb, aa = np.polyfit(np.asarray(sizes, float), np.asarray(ts, float), 1)
            print(json.dumps({"content": content, "form": name, "fixed_us": round(aa * 1e6, 1),
                              "steady_GBps": round(1 / bb / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
