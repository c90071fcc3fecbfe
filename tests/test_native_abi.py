"""CPU checks of the C-ABI library and the product package (no compute calls)."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(REPO, "include", h) for h in ("gmat_hip.h", "gmat_remma_eff.h")]
LIB = os.path.join(REPO, "gmat_amd", "libgmat_hip.so")


def _header_functions():
    names = set()
    for h in HEADERS:
        txt = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"^(?:const\s+)?\w+\s*\*?\s*(\w+)\s*\(", txt, flags=re.M))
    return sorted(names)


def test_library_exports_every_header_symbol():
    if not os.path.exists(LIB):
        pytest.skip("libgmat_hip.so not built")
    lib = ctypes.CDLL(LIB)
    names = _header_functions()
    assert len(names) >= 15
    for name in names:
        assert hasattr(lib, name), name
    from gmat_amd import _native
    assert sorted(_native.exported_symbols()) == names


def test_product_package_does_not_import_oracle():
    code = ("import sys; import gmat_amd, gmat_amd.gmatrix, gmat_amd.uvlmm, gmat_amd.remma, gmat_amd.plink;"
            "bad=[m for m in sys.modules if m=='oracle' or m.startswith('oracle.')];"
            "print(bad); assert not bad")
    subprocess.check_call([sys.executable, "-c", code], cwd=REPO)
    for root, _, files in os.walk(os.path.join(REPO, "gmat_amd")):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(root, f)).read()
                assert "import oracle" not in src and "from oracle" not in src, f


def test_no_gpu_means_loud_failure():
    if not os.path.exists(LIB):
        pytest.skip("libgmat_hip.so not built")
    from gmat_amd import _native
    if _native.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_native.GmatNativeError):
        _native.ensure_device()
