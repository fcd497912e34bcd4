import os, sys, json
import numpy as np
sys.path.insert(0, "/root/repo")
from dataplug_amd import synth
from dataplug_amd.scan import ScanContext
from oracle import dpref
G = 1 << 30
obj = synth.TiledFasta(16 << 30, seed=1)
base = 8 << 30
host = obj.bytes_range(base, base + 4 * G + (64 << 10))
ctx = ScanContext(0)
d = ctx.workspace("in", len(host) + 64)
ctx.h2d(d.ptr, host)
for bb in (0, base):
    for plan_rel in ([(0, G), (G, 2 * G), (2 * G, 3 * G), (3 * G, 4 * G)], [(0, G)], [(0, G), (G, 2 * G)],
                     [(G - (1 << 20), G), (G, G + (1 << 20))], [(0, G), (G, 2 * G), (2 * G, 3 * G)]):
        plan = [(a + bb, b + bb) for a, b in plan_rel]
        exp = dpref.fasta_pairs(host, plan_rel) + np.uint64(bb)
        for u64 in (True, False):
            if not u64 and bb:
                continue
            pairs, pending, cend = ctx.fasta_index(d.ptr, len(host), bb, bb + len(host), plan, u64=u64)
            got = pairs.astype(np.uint64)
            ok = len(got) == len(exp) and np.array_equal(got, exp)
            bad = np.flatnonzero((got != exp).any(axis=1)).tolist()[:3] if len(got) == len(exp) else "count"
            print(json.dumps({"bb": bb, "u64": u64, "plan": [(a - bb, b - bb) for a, b in plan], "ok": bool(ok),
                              "n": len(got), "pending": pending.tolist(), "cend": cend.tolist(), "bad": bad,
                              "bad_vals": [(got[i].tolist(), exp[i].tolist()) for i in bad] if bad != "count" else None}), flush=True)
