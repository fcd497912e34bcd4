"""ISA guard for the hand-waited input loads of scan_kernel (dataplug_amd/csrc/dpscan.hip).

The data waves issue their buffer loads as inline asm and wait with one explicit `s_waitcnt vmcnt(9)`.
The compiler knows nothing about that contract, so this checks the generated gfx950 assembly: on every
control-flow path from a `buffer_load_dword*` into register(s) R to the next `s_waitcnt vmcnt`, no
instruction may read or write R (dataflow over the kernel's basic blocks).  Usage: python tools/isa_guard.py [path/to/dpscan-hip-amdgcn-amd-amdhsa-gfx950.s]
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


BRANCH_RE = re.compile(r"^s_(cbranch_\w+|branch)\s+(\.?\w+)")


def _blocks(body: str):
    """Split a kernel body into basic blocks: (label, [instructions], successors)."""
    blocks, cur, label = [], [], "<entry>"
    for line in body.splitlines():
        s = line.split(";")[0].strip()
        if not s:
            continue
        if s.endswith(":"):
            blocks.append([label, cur])
            label, cur = s[:-1], []
            continue
        cur.append(s)
    blocks.append([label, cur])
    out = []
    for i, (lab, ins) in enumerate(blocks):
        succ = set()
        fall = True
        for s in ins:
            m = BRANCH_RE.match(s)
            if m:
                succ.add(m.group(2))
                if m.group(1) == "branch":
                    fall = False
            if s.split()[0] in ("s_endpgm", "s_setpc_b64"):
                fall = False
        if fall and i + 1 < len(blocks):
            succ.add(blocks[i + 1][0])
        out.append((lab, ins, succ))
    return out


def _scan(ins, pending, problems, k):
    """Run one block: returns the pending set at its end (registers with an un-waited input load)."""
    pending = set(pending)
    for s in ins:
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
            if problems is not None and srcs & pending:
                problems.append((k, s))
            pending |= dst
            continue
        if problems is not None and used & pending:
            problems.append((k, s))
    return pending


def check(asm_path: str):
    """Dataflow over the control-flow graph: a register written by an input buffer load stays "pending" on
    every path until an `s_waitcnt vmcnt`; no instruction on any path may read or write it meanwhile."""
    text = open(asm_path).read()
    problems = []
    kernels = KERNEL_RE.findall(text)
    assert len(kernels) == 4, kernels
    for k in kernels:
        body = text[text.index(k + ":") + len(k) + 1:]
        body = body[:body.index(".Lfunc_end")]
        blocks = _blocks(body)
        index = {lab: i for i, (lab, _, _) in enumerate(blocks)}
        pin = [set() for _ in blocks]
        work = list(range(len(blocks)))
        while work:
            i = work.pop()
            lab, ins, succ = blocks[i]
            pout = _scan(ins, pin[i], None, k)
            for t in succ:
                j = index.get(t)
                if j is not None and not pout <= pin[j]:
                    pin[j] |= pout
                    work.append(j)
        for i, (lab, ins, succ) in enumerate(blocks):
            _scan(ins, pin[i], problems, k)
    return problems


if __name__ == "__main__":
    path = sys.argv[1] if len(sys.argv) > 1 else compile_asm()
    bad = check(path)
    for p in bad[:20]:
        print("touches an un-waited load destination:", p)
    print("ISA guard:", "FAIL" if bad else "ok", len(bad))
    sys.exit(1 if bad else 0)
