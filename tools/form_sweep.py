"""Newline index: the line_kernel and one-pass forms against the read-only stream kernel, alternated rep by rep.

Same box, same resident object (synth.tiled_csv / tiled_vcf of the largest size, uploaded once), every size a
prefix [0, size) of it in the stored form (out_mode 3: uint16 low words + 64 KiB block table).  Every rep runs
the read-only calibration kernel over the same bytes and then each form once (the order rotates per rep), so a
drift of the box touches every form alike; each launch is timed alone (HIP events on the device's scan stream).
Per size: mean / median / min / max of every form, its roofline fraction on algorithmic bytes (N + 2 L + 8 B per
64 KiB block, over 8 TB/s), the stream kernel's, and the shipped default's choice; outputs of all forms compared
byte for byte.

    python tools/form_sweep.py [--content vcf,csv] [--sizes-gib 2,4,8,16,32,64] [--reps 10] [--forms line,one,default]

A form may name its own out_mode (``--forms line:4,one:3,default:4``: 3 uint16 + blocks, 4 uint8 + 256-byte counts +
blocks); forms of one out_mode are compared byte for byte, forms of different modes through the decoded offsets'
count and a checksum of the first and last 1 Mi entries.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd import synth  # noqa: E402
from dataplug_amd.scan import ScanContext  # noqa: E402
from dataplug_amd.scan.objects import BlockedOffsets, ByteOffsets  # noqa: E402

FORM_IDS = {"line": 1, "one": 3, "default": 0}


def make_ctx(form: str) -> ScanContext:
    ctx = ScanContext(0)
    kind = form.split(":")[0]
    if kind != "default":
        ctx.set_form(delim=FORM_IDS[kind])
    return ctx


def form_mode(form: str, default: int) -> int:
    return int(form.split(":")[1]) if ":" in form else default


def alg_bytes(size, n, mode, ntab, nsub):
    return size + (2 if mode == 3 else 1) * n + 8 * ntab + (2 * nsub if mode == 4 else 0)


def stats(ts):
    a = np.asarray(ts, float)
    return {"mean": round(float(a.mean()), 1), "median": round(float(np.median(a)), 1),
            "min": round(float(a.min()), 1), "max": round(float(a.max()), 1), "std": round(float(a.std()), 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--content", default="vcf,csv")
    ap.add_argument("--sizes-gib", default="2,4,8,16,32,64")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--forms", default="line,one,default")
    ap.add_argument("--no-stream", action="store_true")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--begin", type=int, default=0, help="every launch scans [begin, size) of the resident object "
                    "(e.g. 482: a VCF body behind its header, ranges off the 256-byte grid)")
    ap.add_argument("--out-mode", type=int, default=3, choices=[3, 4], help="3: uint16 + blocks, 4: uint8 + 256 B + blocks")
    args = ap.parse_args()
    sizes = [int(float(x) * (1 << 30)) for x in args.sizes_gib.split(",")]
    top = max(sizes)
    names = args.forms.split(",")
    ctxs = {k: make_ctx(k) for k in names}
    ctx0 = next(iter(ctxs.values()))
    d = ctx0.workspace("in", top + 64)
    for content in args.content.split(","):
        t0 = time.perf_counter()
        obj = (synth.tiled_csv if content == "csv" else synth.tiled_vcf)(top, seed=args.seed)
        step = 2 << 30
        stage = np.empty(min(step, top), np.uint8)
        for p in range(0, top, step):
            q = min(top, p + step)
            ctx0.h2d(d.ptr + p, obj.bytes_range(p, q, out=stage))
        del stage
        print(json.dumps({"content": content, "gen_s": round(time.perf_counter() - t0, 2)}), flush=True)
        # every context's output buffer sized for the largest launch once, before any is timed
        top_cap = obj.count_range(0, top) + 1024
        modes = {k: form_mode(k, args.out_mode) for k in names}
        outs = {k: c.workspace("out", ScanContext.out_bytes(top_cap, modes[k], np.asarray([0, top], np.uint64)))
                for k, c in ctxs.items()}
        for size in sizes:
            b0 = args.begin
            n_exp = obj.count_range(b0, size)
            cap = n_exp + 1024
            ranges = np.asarray([b0, size], np.uint64)
            times = {k: [] for k in names}
            chosen = {}
            st = []

            def run(k):
                c = ctxs[k]
                c.delim_ranges_async(d.ptr, top, 0, ranges, 10, 1, 0, 0, outs[k].ptr, modes[k], cap)
                r = c.delim_ranges_result(1)
                if k.startswith("default"):
                    chosen.setdefault(k, []).append(c.last_delim_form())
                return r

            for k in names:                       # warm (code objects, workspace) and the first result
                run(k)
            for c in ctxs.values():
                c.timing(True)
                c.timing_read()
            for rep in range(args.reps):
                if not args.no_stream:
                    ctx0.stream_read(d.ptr, size)
                    ctx0.sync()
                    ms, _ = ctx0.timing_read()
                    st.append(ms * 1e3)
                order = names[rep % len(names):] + names[:rep % len(names)]
                for k in order:
                    n, _, _ = run(k)
                    ms, _ = ctxs[k].timing_read()
                    times[k].append(ms * 1e3)
            for c in ctxs.values():
                c.timing(False)
            res = {}
            for k, c in ctxs.items():
                mode = modes[k]
                words = c.d2h(np.empty(n, np.uint16 if mode == 3 else np.uint8), outs[k].ptr)
                res[k] = (n, words, c.block_table(outs[k].ptr, cap, ranges, mode)) + \
                    ((c.sub_table(outs[k].ptr, cap, ranges),) if mode == 4 else ())
            equal = all(r[0] == n_exp for r in res.values())
            for m in sorted(set(modes.values())):
                same = [res[k] for k in names if modes[k] == m]
                equal = equal and all(all(np.array_equal(x, y) for x, y in zip(same[0][1:], b[1:])) for b in same[1:])
            if len(set(modes.values())) > 1:
                ends = set()
                for k in names:
                    r = res[k]
                    o = ByteOffsets(r[1], r[3], r[2], b0 >> 8, b0 >> 16) if len(r) > 3 else BlockedOffsets(r[1], r[2], b0 >> 16)
                    m = min(n, 1 << 20)
                    ends.add((int(o.to_u64(0, m).sum()), int(o.to_u64(n - m, n).sum())))
                equal = equal and len(ends) == 1
            line = {"content": content, "size_gib": size / (1 << 30), "begin": b0, "seed": args.seed, "out_modes": modes,
                    "entries": n_exp,
                    "equal": bool(equal)}
            if st:
                s = stats(st)
                line["stream_us"] = s
                line["stream_TBps_median"] = round(size / (s["median"] * 1e-6) / 1e12, 3)
            for k in names:
                r = res[k]
                alg = alg_bytes(size - b0, n_exp, modes[k], len(r[2]), len(r[3]) if len(r) > 3 else 0)
                s = stats(times[k])
                line[f"{k}_us"] = s
                line[f"{k}_frac_median"] = round(alg / (s["median"] * 1e-6) / 8e12, 4)
                line[f"{k}_frac_mean"] = round(alg / (s["mean"] * 1e-6) / 8e12, 4)
                if st:
                    line[f"{k}_over_stream"] = round(s["median"] / stats(st)["median"], 4)
                line[f"{k}_all_us"] = [round(t, 1) for t in times[k]]
            for k, v in chosen.items():
                line[f"{k}_forms"] = sorted(set(v))
            print(json.dumps(line), flush=True)
            del res
            if not equal:
                print("MISMATCH", flush=True)
                sys.exit(1)


if __name__ == "__main__":
    main()
