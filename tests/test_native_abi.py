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


def test_text_writers_match_numpy_and_pandas(tmp_path):
    """The host-side text writers (no GPU needed) are byte-identical to np.savetxt and to
    pandas to_csv (CPython float repr) -- the formats of gmatrix.py:10-31."""
    if not os.path.exists(LIB):
        pytest.skip("libgmat_hip.so not built")
    import numpy as np
    import pandas as pd
    from gmat_amd import _native as N
    lib = N.load()
    rng = np.random.default_rng(1)
    vals = np.concatenate([rng.standard_normal(50000) * 10.0 ** rng.integers(-30, 30, 50000),
                           rng.random(20000), np.round(rng.random(5000), 3), [0.0, -0.0, 1e16, 1e15, 1e-4, 1e-5,
                           123456789012345678.0, 5e-324, 1.7976931348623157e308, 0.1, 2.0, -3.5, np.nan, np.inf,
                           -np.inf, 1234567890123456.0, 0.001, 1e22]])
    buf = ctypes.create_string_buffer(64)
    for v in vals.tolist():
        n = lib.gmat_float_repr(v, buf, 64)
        assert buf.value.decode() == repr(v), (v, buf.value)
        assert n == len(repr(v))
    n = 37
    mat = rng.standard_normal((n, n)) * 10.0 ** rng.integers(-8, 8, (n, n))
    mat[3, 2] = 0.0
    p0 = str(tmp_path / "m0")
    assert lib.gmat_write_grm_text(p0.encode(), N.ptr(mat), n, 0, None, 3) == 0
    np.savetxt(str(tmp_path / "e0"), mat)
    assert open(p0, "rb").read() == open(str(tmp_path / "e0"), "rb").read()
    ind = np.tril_indices_from(mat)
    ids = np.array(["id%d" % k for k in range(n)], dtype=object)
    blob = b"".join(s.encode() + b"\0" for s in ids)
    for fmt, a, b in ((1, ind[0] + 1, ind[1] + 1), (2, ids[ind[0]], ids[ind[1]])):
        p = str(tmp_path / ("m%d" % fmt))
        assert lib.gmat_write_grm_text(p.encode(), N.ptr(mat), n, fmt, blob if fmt == 2 else None, 0) == 0
        e = str(tmp_path / ("e%d" % fmt))
        pd.DataFrame({"a": a, "b": b, "v": mat[ind]}).to_csv(e, sep=" ", index=False, header=False)
        assert open(p, "rb").read() == open(e, "rb").read()


def test_hit_row_writer_matches_python_rows(tmp_path):
    """gmat_append_hit_rows (the scans' result files, remma_epiAA.py:84-86 DataFrame.to_csv rows) is
    byte-identical to the Python statement _scan.format_rows, for 3 and 4 value columns, appended
    after existing content, and for zero rows."""
    if not os.path.exists(LIB):
        pytest.skip("libgmat_hip.so not built")
    import numpy as np
    from gmat_amd.remma._scan import append_rows, format_rows
    rng = np.random.default_rng(7)
    n = 3000
    i = np.sort(rng.integers(0, 100000, n)).astype(np.int64)
    j = rng.integers(0, 100000, n).astype(np.int64)
    cols = [rng.standard_normal(n) * 10.0 ** rng.integers(-12, 12, n), rng.random(n) * 40.0,
            rng.random(n) * 10.0 ** rng.integers(-20, -4, n), rng.random(n)]
    cols[0][:6] = [0.0, -0.0, 1e-4, 1e-5, 1e16, 2.0]
    for nf in (3, 4):
        path = str(tmp_path / ("hits%d" % nf))
        with open(path, "w") as f:
            f.write("snp_0 snp_1 eff chi_val p_val\n")
        append_rows(path, [i, j] + cols[:nf], nf)
        append_rows(path, [i[:0], j[:0]] + [c[:0] for c in cols[:nf]], nf)
        with open(path) as f:
            got = f.read()
        assert got == "snp_0 snp_1 eff chi_val p_val\n" + format_rows([i, j] + cols[:nf], nf)
