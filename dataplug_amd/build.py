"""Build libdpscan.so in-tree for gfx950:  python -m dataplug_amd.build"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "dpscan.hip")
OUT = os.path.join(HERE, "lib", "libdpscan.so")
OUT_PROF = os.path.join(HERE, "lib", "libdpscan_prof.so")   # diagnostics: in-kernel section timers
GZ_SRC = os.path.join(HERE, "csrc", "dpgz.c")
GZ_PAR_SRC = os.path.join(HERE, "csrc", "dpgz_par.c")     # parallel inflate of one gzip stream
GZ_OUT = os.path.join(HERE, "lib", "libdpgz.so")            # host-side gzip access-point index (zlib)
ARCH = os.environ.get("DPSCAN_ARCH", "gfx950")


def build(verbose: bool = False, prof: bool = False, defines=(), out=None, src=SRC) -> str:
    out = out or (OUT_PROF if prof else OUT)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-Wno-unused-result", "-o", out + ".tmp", src]
    if prof:
        cmd.insert(1, "-DDP_PROF")
    for d in defines:                      # tuning variants, e.g. DP_RING=5 (tools/probe_perf.py)
        cmd.insert(1, f"-D{d}")
    if verbose:
        cmd.append("-Rpass-analysis=kernel-resource-usage")
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_gz() -> str:
    os.makedirs(os.path.dirname(GZ_OUT), exist_ok=True)
    cc = os.environ.get("CC", "gcc")
    subprocess.run([cc, "-O3", "-fPIC", "-shared", "-Wall", "-Wextra", "-o", GZ_OUT + ".tmp", GZ_SRC, GZ_PAR_SRC,
                    "-lz", "-lpthread"], check=True)
    os.replace(GZ_OUT + ".tmp", GZ_OUT)
    return GZ_OUT


if __name__ == "__main__":
    print(build_gz())
    print(build(verbose="-v" in sys.argv, prof="--prof" in sys.argv))
