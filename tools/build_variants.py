"""Build perf-probe variants of libdpscan.so side by side (dataplug_amd/lib/libdpscan_v_<name>.so).

    python tools/build_variants.py name=DEF1,DEF2=3 name2=DEF3 ...   # '-' for no defines

Variants are diagnostics for same-box comparisons (tools/probe_perf.py with DPSCAN_LIB=...); the shipped
library is always the default build (python -m dataplug_amd.build).
"""
from __future__ import annotations

import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd.build import HERE, build  # noqa: E402


def main(specs):
    jobs = []
    for s in specs:
        name, _, defs = s.partition("=")
        defines = [] if defs in ("", "-") else defs.split(",")
        prof = "DP_PROF" in defines
        defines = [d for d in defines if d != "DP_PROF"]
        out = os.path.join(HERE, "lib", f"libdpscan_v_{name}.so")
        jobs.append((defines, prof, out))
    with ThreadPoolExecutor(4) as ex:
        for out in ex.map(lambda j: build(defines=j[0], prof=j[1], out=j[2]), jobs):
            print(out)


if __name__ == "__main__":
    main(sys.argv[1:])
