import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")
    config.addinivalue_line("markers", "slow: BASELINE-size cases (GiBs)")


@pytest.fixture(scope="session")
def fasta_cases():
    z = np.load(os.path.join(GOLDEN, "fasta_cases.npz"))
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def ctx():
    from dataplug_amd.scan import get_context
    return get_context(0)
