"""The built train kernel keeps the in-gap LDS reads' registers untouched until their wait
(tools/check_asm_rd.py on the gfx950 code object inside libmhppo.so; no GPU needed)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mh-ppo_amd", "mhppo", "lib", "libmhppo.so")


def test_in_gap_lds_reads_are_waited_for():
    if not os.path.exists(LIB):
        pytest.skip("libmhppo.so not built")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_asm_rd.py"), LIB], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 violations" in r.stdout
