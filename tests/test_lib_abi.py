"""The C-ABI library loads on CPU and exports every symbol include/*.h declares."""
import ctypes
import os
import re

from kelpie_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    inc = os.path.join(ROOT, "include")
    for fn in os.listdir(inc):
        if fn.endswith(".h"):
            txt = open(os.path.join(inc, fn)).read()
            syms |= set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(kp_\w+)\s*\(", txt, re.M))
    return syms


def test_every_declared_symbol_is_exported():
    syms = declared_symbols()
    assert {"kp_ctx_create", "kp_posttrain_rank", "kp_all_scores"} <= syms
    L = ctypes.CDLL(_lib.LIB_PATH)
    for s in sorted(syms):
        assert hasattr(L, s), s
    assert set(_lib.EXPORTS) == syms


def test_version_and_errors_without_gpu():
    L = _lib.lib()
    assert b"gfx950" in L.kp_version()
    assert L.kp_posttrain_rank(None, None, None) != 0
