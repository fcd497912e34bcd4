"""Print GPU vs expected for the first failing golden FASTA cases (debug helper, GPU)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dataplug_amd.scan import ScanContext
from oracle import cpu_ref

z = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "fasta_cases.npz"))
ctx = ScanContext(0)
shown = 0
for i in range(len(z["chunk_size"])):
    obj = z["data"][z["data_off"][i]:z["data_off"][i + 1]]
    exp = z["expected"][z["expected_off"][i]:z["expected_off"][i + 1]].reshape(-1, 2)
    plan = cpu_ref.chunk_plan(len(obj), int(z["chunk_size"][i]))
    pairs, pending, cend = ctx.fasta_index_host(obj, 0, len(obj), plan, u64=True)
    if not np.array_equal(pairs.astype(np.int64), exp.astype(np.int64)):
        print("case", i, "size", len(obj), "cs", int(z["chunk_size"][i]), "nchunks", len(plan))
        print("  got", pairs.tolist()[:12])
        print("  exp", exp.tolist()[:12])
        print("  pending", pending.tolist()[:8], "cend", cend.tolist()[:8])
        shown += 1
        if shown >= 6:
            break
