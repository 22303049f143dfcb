"""The C-ABI library loads and exports every symbol include/cvlite.h declares (CPU; no compute)."""
import os
import re

from conftest import ROOT


def test_library_exports_header_symbols():
    from cvlite import _lib
    hdr = open(os.path.join(ROOT, "include", "cvlite.h")).read()
    names = set(re.findall(r"\b(cvl_[a-z0-9_]+)\s*\(", hdr))
    assert names, "no declarations parsed"
    lib = _lib.load()
    for n in sorted(names):
        assert hasattr(lib, n), n
    assert set(_lib.SIGNATURES) == names, sorted(set(_lib.SIGNATURES) ^ names)
    assert lib.cvl_version() >= 100
