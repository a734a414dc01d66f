"""The C-ABI library loads and exports every symbol include/xhe.h declares (CPU-safe)."""
import ctypes
import os
import re

from tests.conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "xhe.h")).read()
    return sorted(set(re.findall(r"\b(xhe_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_binding_table():
    from xfl_amd import _native
    assert sorted(_native.SIGNATURES) == _declared()


def test_library_exports_all_symbols():
    from xfl_amd import _native
    L = ctypes.CDLL(_native.LIB_PATH)
    for name in _declared():
        assert hasattr(L, name), name
    assert b"gfx950" in _native.lib().xhe_version()
