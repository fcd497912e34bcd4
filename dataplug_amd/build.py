"""Build libdpscan.so in-tree for gfx950:  python -m dataplug_amd.build"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "dpscan.hip")
OUT = os.path.join(HERE, "lib", "libdpscan.so")
ARCH = os.environ.get("DPSCAN_ARCH", "gfx950")


def build(verbose: bool = False) -> str:
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-Wno-unused-result", "-o", OUT + ".tmp", SRC]
    if verbose:
        cmd.append("-Rpass-analysis=kernel-resource-usage")
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
