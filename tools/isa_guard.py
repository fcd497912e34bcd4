"""CLI of the ISA guard (the code lives in dataplug_amd/isa_guard.py, which the library build runs):

    python tools/isa_guard.py [path/to/dpscan-hip-amdgcn-amd-amdhsa-gfx950.s]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd.isa_guard import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(sys.argv))
