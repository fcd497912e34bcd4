"""Child process of test_gpu_scan.test_two_processes_one_gpu: K scans on GPU 0 of its own synthetic FASTA
(FASTA and newline index alternating), each checked against the oracle; exits 0 when all are exact."""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd import synth  # noqa: E402
from dataplug_amd.scan import ScanContext  # noqa: E402
from oracle import cpu_ref, dpref  # noqa: E402


def main(seed: int, steps: int) -> int:
    obj = synth.fasta((96 << 20) + 977 * seed, seed)
    plan = cpu_ref.chunk_plan(len(obj), math.ceil(len(obj) / 5))
    exp = dpref.fasta_pairs(obj, plan)
    nl = dpref.delim(obj, 0, len(obj))[0]
    ctx = ScanContext(0)
    try:
        d = ctx.workspace("in", len(obj) + 64)
        ctx.h2d(d.ptr, obj)
        for i in range(steps):
            if i % 2:
                got, _ = ctx.delim_index(d.ptr, len(obj), 0, 0, len(obj), 10)
                assert np.array_equal(got, nl), (seed, i)
            else:
                pairs, pending, _ = ctx.fasta_index(d.ptr, len(obj), 0, len(obj), plan)
                assert (pending == -1).all() and np.array_equal(pairs.astype(np.uint64), exp), (seed, i)
    finally:
        ctx.close()
    print(f"proc {seed}: {steps} scans exact", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(int(sys.argv[1]), int(sys.argv[2])))
