"""The compiled scan kernels honour the hand-waited load contract and spill nothing (tools/isa_guard.py:
dataflow over the gfx950 assembly; no scratch segment).  Compiles dpscan.hip with -save-temps (hipcc
cross-compiles here without a GPU)."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and shutil.which("hipcc") is None,
                    reason="no hipcc")
def test_isa_guard_passes():
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "isa_guard.py")], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ISA guard: ok" in r.stdout
