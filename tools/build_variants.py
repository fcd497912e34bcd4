"""Build perf-probe variants of libdpscan.so side by side (dataplug_amd/lib/libdpscan_v_<name>.so).

    python tools/build_variants.py name=DEF1,DEF2=3 name2=DEF3 ...   # '-' for no defines
    python tools/build_variants.py head@HEAD=- ...                   # the source as of a git revision

Variants are diagnostics for same-box comparisons (tools/gpu_ab.sh with DPSCAN_LIB=...): the diagnostics build
(diag=DP_DIAG: in-kernel realtime stamps for tools/map_timeline.py, place_timeline.py, line_timeline.py) or a
source revision (name@REV).  The shipped library is always the default build (python -m dataplug_amd.build), which
has no switches.
"""
from __future__ import annotations

import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import subprocess  # noqa: E402

from dataplug_amd.build import HERE, SRC, IsaGuardError, build  # noqa: E402


def main(specs):
    jobs = []
    for s in specs:
        name, _, defs = s.partition("=")
        name, _, rev = name.partition("@")
        defines = [] if defs in ("", "-") else defs.split(",")
        diag = "DP_DIAG" in defines
        defines = [d for d in defines if d != "DP_DIAG"]
        out = os.path.join(HERE, "lib", f"libdpscan_v_{name}.so")
        src = SRC
        if rev:                                  # next to the real source so its #include resolves
            src = os.path.join(os.path.dirname(SRC), f"_rev_{name}.hip")
            with open(src, "w") as fh:
                fh.write(subprocess.run(["git", "show", f"{rev}:dataplug_amd/csrc/dpscan.hip"], check=True,
                                        capture_output=True, text=True).stdout)
        jobs.append((defines, diag, out, src))
    # build() runs the ISA guard on each variant's own assembly and installs nothing that fails it: a variant
    # whose compiled code touches an in-flight load destination (or spills) can corrupt addresses and fault the GPU

    def one(j):
        try:
            return build(defines=j[0], diag=j[1], out=j[2], src=j[3])
        except IsaGuardError as e:
            if os.path.exists(j[2]):
                os.remove(j[2])
            return f"REFUSED {j[2]}: {e}"
    with ThreadPoolExecutor(4) as ex:
        for out in ex.map(one, jobs):
            print(out)
    for j in jobs:
        if j[3] != SRC:
            os.remove(j[3])


if __name__ == "__main__":
    main(sys.argv[1:])
