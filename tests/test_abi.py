"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports
every entry point include/ipmz.h declares, and fails loudly (no CPU
fallback) when no gfx950 device is visible."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ipmz.h")
LIB = os.path.join(REPO, "ipm-zoo_amd", "lib", "libipmz.so")


def declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ipmz_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_boundary():
    names = declared()
    for must in ("ipmz_ldlt_decomposition", "ipmz_overwriting_solve_ldlt", "ipmz_ldlt_factor", "ipmz_ldlt_solve",
                 "ipmz_qp_create", "ipmz_qp_load_host", "ipmz_qp_step", "ipmz_qp_solve"):
        assert must in names


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build first: __graft_entry__.build()"
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_lists_every_export():
    import ipmz_amd
    assert sorted(ipmz_amd.EXPORTS) == declared()


def test_no_cpu_fallback_without_device():
    import ipmz_amd
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible")
    except ImportError:
        pass
    with pytest.raises(ipmz_amd.IpmzError, match="no gfx950 device"):
        ipmz_amd.Context(0)


def test_product_does_not_reference_oracle():
    # the product path must not route through the CPU oracle
    pkg = os.path.join(REPO, "ipm-zoo_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h", ".hpp")):
                txt = open(os.path.join(root, f), errors="replace").read()
                assert "libipmz_oracle" not in txt and "import oracle" not in txt and "ipmzo_" not in txt, f
