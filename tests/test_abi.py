"""The C-ABI library loads and exports every symbol include/mhppo.h declares (no GPU needed)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mhppo.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mhppo_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared()
    assert "mhppo_env_step" in names and "mhppo_returns_scan" in names


def test_library_exports_all_declared_symbols():
    from mhppo import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"{_lib.LIB_PATH} not built (run __graft_entry__.build())")
    so = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared() if not hasattr(so, n)]
    assert not missing, f"libmhppo.so lacks: {missing}"


def test_binding_covers_header():
    from mhppo import _lib
    assert set(_lib.declared_symbols()) <= set(declared())
