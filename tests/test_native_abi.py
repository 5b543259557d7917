"""CPU-side checks of the C ABI boundary: the library loads (no GPU needed to dlopen) and exports every entry
point that include/arcweld_amd.h declares; the Python binding covers all of them."""
import os
import re

from conftest import REPO


def _declared():
    src = open(os.path.join(REPO, "include", "arcweld_amd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(aw_\w+)\s*\(", src, re.M)))


def test_header_declares_entry_points():
    names = _declared()
    assert "aw_gemm" in names and "aw_vq_forward" in names and len(names) >= 25


def test_library_exports_every_declared_symbol():
    from arcweld import _native
    lib = _native.load()
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_every_declared_symbol():
    from arcweld import _native
    missing = [n for n in _declared() if n not in _native.SIGNATURES and n != "aw_last_error"]
    assert not missing, missing


def test_cpu_tensors_are_rejected():
    import pytest
    import torch
    from arcweld import _native
    with pytest.raises(_native.NativeError):
        _native.ptr(torch.zeros(3))
