"""Build libdpscan.so in-tree for gfx950:  python -m dataplug_amd.build

The scan library is compiled with -save-temps and the ISA guard (dataplug_amd/isa_guard.py) checks that exact
device assembly: every kernel, no touched in-flight load destination, no scratch segment.  Only a library that
passes is installed (os.replace after the guard), next to a stamp ``<lib>.isa.json`` holding the guard's report
and the installed file's sha256; the loader (scan/_lib.py) refuses a library whose stamp is missing, failed or
belongs to another file.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

from dataplug_amd import isa_guard

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "dpscan.hip")
OUT = os.path.join(HERE, "lib", "libdpscan.so")
OUT_DIAG = os.path.join(HERE, "lib", "libdpscan_diag.so")   # diagnostics: in-kernel realtime stamps (-DDP_DIAG)
GZ_SRC = os.path.join(HERE, "csrc", "dpgz.c")
GZ_PAR_SRC = os.path.join(HERE, "csrc", "dpgz_par.c")     # parallel inflate of one gzip stream
GZ_OUT = os.path.join(HERE, "lib", "libdpgz.so")            # host-side gzip access-point index (zlib)
ARCH = os.environ.get("DPSCAN_ARCH", "gfx950")


class IsaGuardError(RuntimeError):
    """The compiled kernels fail the ISA guard: the library is not installed."""


def sha256_file(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def stamp_path(lib: str) -> str:
    return lib + ".isa.json"


def build(verbose: bool = False, diag: bool = False, defines=(), out=None, src=SRC) -> str:
    """Compile ``src`` for gfx950, run the ISA guard on its assembly, install it at ``out`` only if it passes.
    The shipped library has no defines; ``diag`` builds the diagnostics library (-DDP_DIAG: in-kernel realtime
    stamps, lib/libdpscan_diag.so), guarded like the shipped one and loaded only through DPSCAN_LIB."""
    out = out or (OUT_DIAG if diag else OUT)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    defs = (["DP_DIAG"] if diag else []) + list(defines)
    with tempfile.TemporaryDirectory(prefix="dpscan_build_") as d:
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
               "-Wno-unused-result", "-save-temps"] + [f"-D{x}" for x in defs] + ["-o", os.path.join(d, "lib.so"),
                                                                                  os.path.abspath(src)]
        if verbose:
            cmd.append("-Rpass-analysis=kernel-resource-usage")
        subprocess.run(cmd, check=True, cwd=d)
        stem = os.path.splitext(os.path.basename(src))[0]
        asm = os.path.join(d, f"{stem}-hip-amdgcn-amd-amdhsa-{ARCH}.s")
        rep = isa_guard.verify(asm)
        print(f"ISA guard: {rep['result']} ({len(rep['kernels'])} kernels, {os.path.basename(out)})",
              file=sys.stderr if rep["result"] != "ok" else sys.stdout, flush=True)
        if rep["result"] != "ok":
            raise IsaGuardError(f"{out} not installed: the ISA guard failed on its assembly: "
                                f"{rep['violations'][:3]} {rep['scratch'][:3]} missing {rep['missing_kernels']}")
        shutil.copyfile(os.path.join(d, "lib.so"), out + ".tmp")
        rep.update(so_sha256=sha256_file(out + ".tmp"), asm_sha256=sha256_file(asm), defines=defs, arch=ARCH,
                   source=os.path.relpath(os.path.abspath(src), os.path.dirname(HERE)), src_sha256=sha256_file(src),
                   guard_enforced=True)
        with open(stamp_path(out) + ".tmp", "w") as f:
            json.dump(rep, f, indent=1)
        os.replace(stamp_path(out) + ".tmp", stamp_path(out))
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
    print(build(verbose="-v" in sys.argv, diag="--diag" in sys.argv))
