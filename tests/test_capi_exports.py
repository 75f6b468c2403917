"""CPU: the C-ABI library loads and exports exactly what include/mlamg.h declares (no GPU calls)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mlamg.h")
LIB = os.path.join(ROOT, "ml-amg_amd", "mlamg", "libmlamg_hip.so")


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mlamg_[A-Za-z0-9_]+)\s*\(", src)))


def test_header_parses():
    syms = header_symbols()
    assert "mlamg_spmv" in syms and "mlamg_hier_vcycle" in syms
    assert len(syms) >= 40


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmlamg_hip.so not built")
def test_library_exports_every_header_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, f"not exported: {missing}"


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmlamg_hip.so not built")
def test_python_binding_covers_header():
    from mlamg import _lib
    assert set(_lib.SIGNATURES) == set(header_symbols())
    assert _lib.lib.mlamg_version() >= 10000


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmlamg_hip.so not built")
def test_errors_are_reported_without_gpu():
    from mlamg import _lib
    # argument validation happens before any device call
    rc = _lib.lib.mlamg_spmv(None, None, None, 1.0, 0.0, None)
    assert rc == _lib.MLAMG_EINVAL
    assert b"NULL" in _lib.lib.mlamg_last_error()
    with pytest.raises(_lib.MlamgError):
        _lib.call("mlamg_hier_set_smoothing", None, 1, 1)
