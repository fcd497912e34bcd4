"""ISA guard for the hand-waited loads of libdpscan's kernels (dataplug_amd/csrc/dpscan.hip).

``dataplug_amd.build.build()`` runs it on the exact assembly of the library it builds (-save-temps) and installs
the library only if it passes (round 3's GPU fault came from a variant that failed it and was run anyway).

The data waves issue their buffer loads as inline asm and wait with one explicit `s_waitcnt vmcnt(N)` per
buffer, N = the loads of the buffers still in flight.  The compiler knows nothing about that contract, so
this checks the generated gfx950 assembly: on every control-flow path from a `buffer_load_dword*` (or a
returning `buffer_atomic_* … sc0`) into register(s) R until a wait that the load is certain to have completed by (vmcnt(N) with fewer than N
vector-memory operations issued after it), no instruction may read or write R (dataflow over the
kernel's basic blocks, tracking the ordered queue of outstanding vector-memory operations).  Every kernel of the
code object is checked (the scans, the map and placement kernels, the density probe, resolve/find and the calibration kernels), and
the check fails if any kernel has a scratch segment (register spills or private arrays in memory).

    python -m dataplug_amd.isa_guard [path/to/dpscan-hip-amdgcn-amd-amdhsa-gfx950.s]

(without an argument it compiles the kernel with -save-temps into a temp dir; DP_DEFINES=A=1,B adds -D's).
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

SRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc", "dpscan.hip")
# every kernel symbol of the device assembly (anonymous-namespace kernels: _ZN12_GLOBAL__N_1<len><name>...)
KERNEL_RE = re.compile(r"^(_ZN12_GLOBAL__N_1\d+\w+?_kernel\w*):", re.M)
# kernels the shipped library must contain (a build that lost one is not the library the tests describe)
REQUIRED = ("scan_kernel", "map_kernel", "fasta_place_kernel", "line_kernel",
            "density_probe_kernel", "fasta_resolve_kernel", "find_kernel", "stream_kernel", "stream_rw_kernel")


def compile_asm() -> str:
    d = tempfile.mkdtemp(prefix="dpscan_isa_")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-Wno-unused-function", "-save-temps", "-o", os.path.join(d, "x.so"), SRC]
                   + ["-D" + x for x in os.environ.get("DP_DEFINES", "").split(",") if x], cwd=d, check=True,
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
    in_asm = False
    for line in body.splitlines():
        if "#ASMSTART" in line:
            in_asm = True
        elif "#ASMEND" in line:
            in_asm = False
        s = line.split(";")[0].strip()
        if not s:
            continue
        if in_asm and not s.endswith(":"):
            s += " @asm"                          # written by hand (inline asm), not by the compiler
            if "dp_win_read" in line:
                s += " @winread"                  # an LDS read of line_kernel's LDS-DMA look-back window
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


VMEM_RE = re.compile(r"^(buffer|global|flat|scratch)_(load|store|atomic)")
VMCNT_RE = re.compile(r"vmcnt\((\d+)\)")
MAXQ = 64          # the vmcnt counter's range: older operations have completed


def _join(a, b):
    n = max(len(a), len(b))
    e = frozenset()
    return tuple((a[i] if i < len(a) else e) | (b[i] if i < len(b) else e) for i in range(n))


def _le(a, b):
    return len(a) <= len(b) and all(x <= b[i] for i, x in enumerate(a))


def _scan(ins, q, problems, k):
    """Run one block over q, the outstanding vector-memory operations youngest first (vmcnt decrements
    in issue order): each entry is the set of VGPRs an input buffer load will still write (empty for
    any other load/store, which only takes a counter slot; {"lds"} for an LDS-DMA load, whose destination is
    LDS).  `s_waitcnt vmcnt(N)` keeps the N youngest.  An LDS read tagged `dp_win_read` (line_kernel's
    look-back window) is a violation while any LDS-DMA load may still be outstanding: it would read another
    group's or a partial window."""
    q = tuple(q)
    for s in ins:
        toks = re.split(r"[\s,]+", s)
        op = toks[0]
        if op == "s_waitcnt":
            m = VMCNT_RE.search(s)
            if m:
                q = q[:int(m.group(1))]
            continue
        pending = frozenset().union(*q) if q else frozenset()
        if "@winread" in toks and "lds" in pending:
            if problems is not None:
                problems.append((k, s))
        if VMEM_RE.match(op):
            # hand-waited destinations: the input buffer loads and the returning (sc0) ticket atomic
            # (global atomics: only the inline-asm claims are hand-waited; the compiler waits for its own)
            # (and inline-asm global loads: line_kernel's look-back descriptors, read after a later buffer wait)
            if op.startswith("buffer_load_dword") or (op.startswith("buffer_atomic") and "sc0" in toks[1:]) or \
                    (op.startswith("global_atomic") and "sc0" in toks[1:] and "@asm" in toks[1:]) or \
                    (op.startswith("global_load") and "@asm" in toks[1:]):
                dst = {"lds"} if "_lds" in op else regs(toks[1])   # LDS-DMA: no VGPR destination, LDS pending
                srcs = set()
                for t in toks[2:]:
                    srcs |= regs(t)
                if problems is not None and srcs & pending:
                    problems.append((k, s))
                q = ((frozenset(dst),) + q)[:MAXQ]
            else:
                used = set()
                for t in toks[1:]:
                    used |= regs(t)
                if problems is not None and used & pending:
                    problems.append((k, s))
                q = ((frozenset(),) + q)[:MAXQ]
            continue
        used = set()
        for t in toks[1:]:
            used |= regs(t)
        if problems is not None and used & pending:
            problems.append((k, s))
    return q


def check(asm_path: str):
    """Dataflow over the control-flow graph: a register written by an input buffer load stays "pending" on
    every path until a `s_waitcnt vmcnt(N)` with fewer than N vector-memory operations issued after the
    load; no instruction on any path may read or write it meanwhile."""
    text = open(asm_path).read()
    problems = []
    kernels = KERNEL_RE.findall(text)
    for k in kernels:
        body = text[text.index(k + ":") + len(k) + 1:]
        body = body[:body.index(".Lfunc_end")]
        blocks = _blocks(body)
        index = {lab: i for i, (lab, _, _) in enumerate(blocks)}
        pin = [() for _ in blocks]
        work = list(range(len(blocks)))
        while work:
            i = work.pop()
            lab, ins, succ = blocks[i]
            pout = _scan(ins, pin[i], None, k)
            for t in succ:
                j = index.get(t)
                if j is not None and not _le(pout, pin[j]):
                    pin[j] = _join(pin[j], pout)
                    work.append(j)
        for i, (lab, ins, succ) in enumerate(blocks):
            _scan(ins, pin[i], problems, k)
    return problems


def kernel_names(asm_path: str):
    return KERNEL_RE.findall(open(asm_path).read())


def short_name(sym: str) -> str:
    """_ZN12_GLOBAL__N_111scan_kernelILi1ELi2EE... -> scan_kernel<1,2>"""
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", sym)
    n = int(m.group(1))
    base = sym[m.end():m.end() + n]
    targs = re.match(r"I((?:Li\d+E)+)E", sym[m.end() + n:])
    if not targs:
        return base
    return base + "<" + ",".join(re.findall(r"Li(\d+)E", targs.group(1))) + ">"


def verify(asm_path: str) -> dict:
    """The guard's verdict on one assembly file: every kernel checked, the violations and scratch segments."""
    kernels = kernel_names(asm_path)
    bad = check(asm_path)
    spills = scratch(asm_path)
    names = [short_name(k) for k in kernels]
    missing = [r for r in REQUIRED if not any(n.split("<")[0] == r for n in names)]
    ok = not bad and not spills and not missing
    return {"result": "ok" if ok else "FAIL", "kernels": names,
            "violations": [f"{short_name(k)}: {s}" for k, s in bad[:20]], "n_violations": len(bad),
            "scratch": [f"{short_name(k)}: {n} B per lane" for k, n in spills], "missing_kernels": missing}


def scratch(asm_path: str):
    """Kernels with a private (scratch) segment: register spills or private arrays in memory.  A spill reload in
    the coordinator queues behind the CU's input stream (8 look-back windows did this: FASTA -2 %); a private
    array in the placement kernel forced a wait on its prefetched spill words (round 3)."""
    text = open(asm_path).read()
    out = []
    for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", text, re.S):
        sz = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", m.group(2))
        if sz and int(sz.group(1)) > 0:
            out.append((m.group(1), int(sz.group(1))))
    return out


def main(argv) -> int:
    path = argv[1] if len(argv) > 1 else compile_asm()
    rep = verify(path)
    for p in rep["violations"]:
        print("touches an un-waited load destination:", p)
    for p in rep["scratch"]:
        print("scratch segment (register spills):", p)
    for p in rep["missing_kernels"]:
        print("kernel missing from the code object:", p)
    print(f"ISA guard: {rep['result']} ({len(rep['kernels'])} kernels, "
          f"{rep['n_violations'] + len(rep['scratch']) + len(rep['missing_kernels'])} problems)")
    return 0 if rep["result"] == "ok" else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv))
