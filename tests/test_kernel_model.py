"""Lane-exact numpy model of scan_kernel (tools/emulate_kernel.py) vs the oracle: the kernel's bit
formulas, ballots, unit geometry and look-back composition, checked on CPU at small sizes."""
import os
import sys

import numpy as np
import pytest

from oracle import cpu_ref, dpref

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import emulate_kernel as emu  # noqa: E402


def _adversarial(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "random":
        return rng.choice(np.frombuffer(b">\nA", np.uint8), size=n, p=[0.05, 0.1, 0.85])
    if kind == "dense":
        return rng.choice(np.frombuffer(b">\n", np.uint8), size=n)
    if kind == "long_lines":
        return rng.choice(np.frombuffer(b">\nA", np.uint8), size=n, p=[0.001, 0.0005, 0.9985])
    raise ValueError(kind)


@pytest.mark.parametrize("kind,n,div", [("random", 40_000, 1), ("random", 300_000, 3), ("dense", 150_000, 7),
                                        ("long_lines", 200_000, 2)])
def test_model_fasta_matches_oracle(kind, n, div):
    a = _adversarial(kind, n, n + div)
    cs = max(1, n // div)
    plan = cpu_ref.chunk_plan(n, cs)
    exp = dpref.fasta_pairs(a, plan)
    got = emu.run(a, plan, "fasta")
    assert np.array_equal(got.astype(np.uint64), exp)


@pytest.mark.parametrize("every_k,emit_add,begin,end", [(1, 0, 0, 200_000), (4, 1, 3, 199_990), (2, 5, 70_000, 70_001)])
def test_model_delim_matches_oracle(every_k, emit_add, begin, end):
    a = _adversarial("random", 200_000, every_k)
    got = emu.run(a, [(begin, end)], "delim", every_k=every_k, emit_add=emit_add)
    exp = cpu_ref.delim_index(a, begin, end, 10, every_k, emit_add)
    assert np.array_equal(got.astype(np.uint64), exp)
