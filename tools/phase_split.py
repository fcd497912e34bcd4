"""Split a rocprofv3 kernel trace of bench.py into its phases (profiles/<tag>/scan_launches_by_phase.json).

    python tools/phase_split.py gpurun_out/prof_<tag> profiles/<tag> --warmup W --steps K [--mode 0|1]

bench.py launches the scan max(2, W) times untimed, then K times with HIP events around each launch (the
roofline phase), K times serialized (the secondary `serialized` field) and K times pipelined (the `value`
phase).  rocprofv3's --stats average mixes all of them; the roofline-phase average is the one that must
agree with bench.py's `roofline.kernel_avg_us`.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--mode", default="0", help="scan_kernel template mode: 0 FASTA, 1 DELIM")
    args = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(args.src, "trace", "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            if f"scan_kernel<{args.mode}," in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    dur = [(e - s) / 1e3 for s, e in rows]
    w = max(2, args.warmup)
    K = args.steps
    phases = {"warmup": dur[:w], "events (roofline phase)": dur[w:w + K],
              "serialized": dur[w + K:w + 2 * K], "pipelined (value phase)": dur[w + 2 * K:w + 3 * K]}
    out = {k: {"launches": len(v), "avg_us": round(sum(v) / len(v), 1), "min_us": round(min(v), 1),
               "max_us": round(max(v), 1)} for k, v in phases.items() if v}
    out["all"] = {"launches": len(dur), "avg_us": round(sum(dur) / max(1, len(dur)), 1)}
    log = os.path.join(args.src, "trace.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{"):
                out["bench_under_rocprof_kernel_avg_us"] = json.loads(line)["roofline"]["kernel_avg_us"]
    out["source"] = (f"{args.src}/trace/*kernel_trace.csv (launches 0-{w - 1} warmup, {w}-{w + K - 1} with events, "
                     f"{w + K}-{w + 2 * K - 1} serialized, {w + 2 * K}-{w + 3 * K - 1} pipelined)")
    os.makedirs(args.dst, exist_ok=True)
    with open(os.path.join(args.dst, "scan_launches_by_phase.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
