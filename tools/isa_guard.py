"""ISA guard for the hand-waited input loads of scan_kernel (dataplug_amd/csrc/dpscan.hip).

The data waves issue their buffer loads as inline asm and wait with one explicit `s_waitcnt vmcnt(9)`.
The compiler knows nothing about that contract, so this checks the generated gfx950 assembly: between a
`buffer_load_dword*` into register(s) R and the next `s_waitcnt vmcnt`, no instruction may read or write
R.  Usage: python tools/isa_guard.py [path/to/dpscan-hip-amdgcn-amd-amdhsa-gfx950.s]
(without an argument it compiles the kernel with -save-temps into a temp dir).
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "dataplug_amd", "csrc", "dpscan.hip")
KERNEL_RE = re.compile(r"^(_ZN12_GLOBAL__N_111scan_kernelILi[01]ELi[01]EE\w*):", re.M)


def compile_asm() -> str:
    d = tempfile.mkdtemp(prefix="dpscan_isa_")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-Wno-unused-function", "-save-temps", "-o", os.path.join(d, "x.so"), SRC], cwd=d, check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return os.path.join(d, "dpscan-hip-amdgcn-amd-amdhsa-gfx950.s")


def regs(tok: str):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()


def check(asm_path: str):
    text = open(asm_path).read()
    problems = []
    kernels = KERNEL_RE.findall(text)
    assert len(kernels) == 4, kernels
    for k in kernels:
        body = text[text.index(k + ":"):]
        body = body[:body.index(".Lfunc_end")]
        pending = set()          # registers with an un-waited input load
        prev_uncond = False
        for ln, line in enumerate(body.splitlines()):
            s = line.split(";")[0].strip()
            if not s:
                continue
            if s.endswith(":"):
                # conservative: a block can be entered from anywhere, so pending loads stay pending
                # until a vmcnt wait (textual order; may over-report, never under-reports a path the
                # layout puts after the loads)
                continue
            prev_uncond = s.split()[0] in ("s_branch", "s_endpgm", "s_setpc_b64")
            if s.startswith("s_waitcnt") and "vmcnt" in s:
                pending.clear()
                continue
            toks = re.split(r"[\s,]+", s)
            used = set()
            for t in toks[1:]:
                used |= regs(t)
            if toks[0].startswith("buffer_load_dword"):
                dst = regs(toks[1])
                srcs = set()
                for t in toks[2:]:
                    srcs |= regs(t)
                if srcs & pending:
                    problems.append((k, ln, s))
                pending |= dst
                continue
            if used & pending:
                problems.append((k, ln, s))
    return problems


if __name__ == "__main__":
    path = sys.argv[1] if len(sys.argv) > 1 else compile_asm()
    bad = check(path)
    for p in bad[:20]:
        print("touches an un-waited load destination:", p)
    print("ISA guard:", "FAIL" if bad else "ok", len(bad))
    sys.exit(1 if bad else 0)
