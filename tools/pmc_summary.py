"""Summarise a tools/profile.sh run into per-launch numbers for one kernel (profiles/<tag>/pmc_summary.json).

    python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<tag> [--kernel scan_kernel<0>|fasta_map_kernel,fasta_place_kernel]

Counters are averaged over the kernel's dispatches, summed over the per-XCD/SE rows rocprofv3 reports per
dispatch.  FETCH_SIZE/WRITE_SIZE are in KB (1024 B); on gfx950 FETCH_SIZE counts half of the wide
streaming reads (MI355X_MICROARCH.md HBM/rocprofv3 section), so HBM read bytes = 2 x FETCH_SIZE x 1024.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
from collections import defaultdict


def split_kernels(kernel: str):
    """Comma-separated kernel names, commas inside template brackets kept ("scan_kernel<1, 2>" is one name)."""
    out, depth, cur = [], 0, ""
    for ch in kernel:
        depth += (ch == "<") - (ch == ">")
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    return out + [cur]


def counters(path: str, kernel: str):
    """Per-dispatch averages of each counter for one kernel name, or the SUM of those averages over a
    comma-separated list of kernels that make up one launch (the FASTA map + placement kernels)."""
    out = defaultdict(float)
    for k in split_kernels(kernel):
        per = defaultdict(lambda: defaultdict(float))
        for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if k in row["Kernel_Name"]:
                    per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
        for c, d in per.items():
            if d:
                out[c] += sum(d.values()) / len(d)
    return dict(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--kernel", default="scan_kernel<0>")
    ap.add_argument("--alg-bytes", type=float, default=None)
    ap.add_argument("--object-bytes", type=int, default=None, help="scanned bytes per launch (bench.py checks it)")
    ap.add_argument("--index-dtype", default=None, help="csv/vcf index form profiled (bench.py checks it)")
    args = ap.parse_args()
    os.makedirs(args.dst, exist_ok=True)
    out = counters(args.src, args.kernel)
    if "FETCH_SIZE" in out:
        out["hbm_read_bytes_corrected"] = out["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in out:
        out["hbm_write_bytes"] = out["WRITE_SIZE"] * 1024
    if "hbm_read_bytes_corrected" in out and "hbm_write_bytes" in out:
        out["hbm_traffic_bytes"] = out["hbm_read_bytes_corrected"] + out["hbm_write_bytes"]
    if args.alg_bytes:
        out["alg_bytes"] = args.alg_bytes
        if "hbm_traffic_bytes" in out:
            out["traffic_over_alg"] = out["hbm_traffic_bytes"] / args.alg_bytes
    out["kernel"] = args.kernel
    if args.object_bytes:
        out["object_bytes"] = args.object_bytes
    if args.index_dtype:
        out["index_dtype"] = args.index_dtype
    for f in glob.glob(os.path.join(args.src, "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(args.dst, "kernel_stats.csv"))
    for f in glob.glob(os.path.join(args.src, "*.log")):
        if os.path.basename(f).startswith("trace"):
            shutil.copy(f, os.path.join(args.dst, "bench_under_rocprof.log"))
    with open(os.path.join(args.dst, "pmc_summary.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
