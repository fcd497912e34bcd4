"""Per-kernel summary of a tools/kernel_pmc.sh run: every kernel's average duration (kernel trace) and its SQ
counters per dispatch (summed over the per-XCD/SE rows rocprofv3 reports), with instruction counts per wave and
the wait counters as shares of SQ_WAVE_CYCLES.

    python tools/kernel_pmc.py gpurun_out/kpmc_<tag>
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0]


def main(src):
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))   # kernel -> counter -> dispatch -> value
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            per[short(row["Kernel_Name"])][row["Counter_Name"]][(f, row["Dispatch_Id"])] += float(row["Counter_Value"])
    dur = {}
    for f in glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            dur[short(row["Name"])] = (int(row["Calls"]), float(row["AverageNs"]) / 1e3)
    out = {}
    for k in sorted(set(per) | set(dur)):
        c = {n: sum(d.values()) / len(d) for n, d in per[k].items() if d}
        r = {"calls": dur.get(k, (None, None))[0], "avg_us": dur.get(k, (None, None))[1]}
        waves = c.get("SQ_WAVES") or None
        cyc = c.get("SQ_WAVE_CYCLES") or None
        for n, v in sorted(c.items()):
            if n.startswith("SQ_INSTS") and waves:
                r[n + "_per_wave"] = round(v / waves, 1)
            elif n.startswith(("SQ_WAIT", "SQ_ACTIVE")) and cyc:
                r[n + "_share"] = round(v / cyc, 3)
            else:
                r[n] = round(v, 1)
        out[k] = r
        print(json.dumps({"kernel": k, **r}))
    with open(os.path.join(src, "kernel_pmc.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
