"""Short randomized parity campaigns on the GPU (tools/fuzz_gpu.py), so every GPU test run also draws fresh
random cases: the kernels through the C ABI against the C oracle, and co.preprocess() end to end with the
multi-group split, launch budgets and the joblib route.  The long campaigns and their logs are in
profiles/r02/fuzz_*.  A failing case is kept in gpurun_out/fuzz_fail.npz."""
import os
import sys
import types

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

pytestmark = pytest.mark.gpu


def _args(seconds, max_size):
    return types.SimpleNamespace(seconds=seconds, max_size=max_size)


def test_fuzz_kernels_vs_oracle():
    import fuzz_gpu
    seed = int.from_bytes(os.urandom(4), "little")
    print(f"seed {seed}")
    st = fuzz_gpu.kernel_mode(_args(12, 8 << 20), np.random.default_rng(seed))
    assert st["fasta_cases"] > 10 and st["delim_cases"] > 10


def test_fuzz_preprocess_groups_vs_oracle():
    import fuzz_gpu
    seed = int.from_bytes(os.urandom(4), "little")
    print(f"seed {seed}")
    st = fuzz_gpu.object_mode(_args(12, 4 << 20), np.random.default_rng(seed))
    assert st["object_cases"] > 10
