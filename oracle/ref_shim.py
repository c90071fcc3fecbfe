"""Container-only loader that imports the REFERENCE GMAT package from /root/reference.

TEST INFRASTRUCTURE ONLY -- never imported by gmat_amd, bench.py's timed path or the
GPU box (where /root/reference does not exist).  It exists to generate the golden
fixtures under tests/golden/ (see tests/golden/make_golden.py) by running the
reference's own code.

Three pieces the reference needs are absent from this image:

1. ``pandas_plink`` (3rd-party, pinned only as ``>=2.0.0`` at setup.py:21, not
   installed).  It is replaced by an in-memory module whose ``read_plink1_bin`` runs
   the reference's OWN C decoder ``read_plink_bed`` (gmat/process_plink/_read_plink_bed.c:5-51,
   compiled unmodified by oracle/Makefile into oracle/_ref/libreadbed.so) and maps the
   missing code 1/3 to NaN exactly as ``Bed.read`` does (read_plink_bed.py:19-28).
   Allele orientation: the C decoder counts the second .bim allele (code 11 -> 2),
   which is pandas_plink's default ``ref="a1"`` orientation.
2. the cffi modules ``_cremma_epi_eff_cpu`` / ``_cread_plink_bed`` (cffi is not importable
   here).  They are replaced by ctypes bindings of the same reference C sources with the
   prototypes of gmat/remma/_build.py:8-31 and a pass-through ``ffi``.
3. ``np.int`` (removed in numpy 1.24, used at remma_epiAA_pair.py:75 and
   random_pair.py:33) is aliased to ``int``.
"""
import ctypes
import os
import subprocess
import sys
import types

import numpy as np

REF_ROOT = "/root/reference"
_HERE = os.path.dirname(os.path.abspath(__file__))
_REF_LIB = os.path.join(_HERE, "_ref")

_LL = ctypes.c_longlong
_PLL = ctypes.POINTER(ctypes.c_longlong)
_PD = ctypes.POINTER(ctypes.c_double)


def build_ref_libs():
    if not (os.path.exists(os.path.join(_REF_LIB, "libremma_epi.so"))
            and os.path.exists(os.path.join(_REF_LIB, "libreadbed.so"))):
        subprocess.check_call(["make", "-s", "-C", _HERE])


class _Ffi:
    """Pass-through stand-in for the cffi ``ffi`` object used by the reference wrappers."""

    def new(self, ctype, init=None):
        if ctype.startswith("char"):
            return ctypes.create_string_buffer(init)
        raise NotImplementedError(ctype)

    def cast(self, ctype, val):
        if ctype == "long long":
            return _LL(int(val))
        if ctype == "double":
            return ctypes.c_double(float(val))
        if ctype.endswith("*"):
            if isinstance(val, int):  # a raw address (ndarray.ctypes.data)
                return ctypes.cast(val, _PD if ctype.startswith("double") else _PLL)
            return val
        raise NotImplementedError(ctype)

    def from_buffer(self, arr):
        return arr


def _as_ptr(arr, ptype):
    if isinstance(arr, np.ndarray):
        return arr.ctypes.data_as(ptype)
    return arr


class _EffLib:
    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, name):
        fn = getattr(self._lib, name)

        def call(*args):
            conv = []
            for a in args:
                if isinstance(a, np.ndarray):
                    conv.append(a.ctypes.data_as(_PD if a.dtype == np.float64 else _PLL))
                elif isinstance(a, int):
                    conv.append(_LL(a))
                elif isinstance(a, float):
                    conv.append(ctypes.c_double(a))
                else:
                    conv.append(a)
            return fn(*conv)
        return call


def _read_plink1_bin(bed, bim, fam, verbose=False, ref="a1"):
    """In-memory pandas_plink stand-in backed by the reference's C decoder."""
    prefix = bed[:-4]
    n = sum(1 for _ in open(fam))
    m = sum(1 for _ in open(bim))
    lib = ctypes.CDLL(os.path.join(_REF_LIB, "libreadbed.so"))
    lib.read_plink_bed.argtypes = [ctypes.c_char_p, _LL, _LL, _PD]
    mat = np.ones(n * m, dtype=np.float64)
    lib.read_plink_bed(prefix.encode("ascii"), n, m, mat.ctypes.data_as(_PD))
    mat[np.abs(mat - 1.0 / 3) < 0.0001] = np.nan
    mat.shape = (m, n)
    ns = types.SimpleNamespace()
    ns.values = np.ascontiguousarray(mat.T)
    return ns


def import_reference():
    """Install the shims and import ``gmat`` from /root/reference.  Returns the module."""
    build_ref_libs()
    if not hasattr(np, "int"):
        np.int = int  # noqa: reference uses np.int (remma_epiAA_pair.py:75, random_pair.py:33)
    pp = types.ModuleType("pandas_plink")
    pp.read_plink1_bin = _read_plink1_bin
    sys.modules["pandas_plink"] = pp

    epi = ctypes.CDLL(os.path.join(_REF_LIB, "libremma_epi.so"))
    for name in ("remma_epiAA_eff_cpu", "remma_epiAD_eff_cpu", "remma_epiDD_eff_cpu"):
        getattr(epi, name).argtypes = [ctypes.c_char_p, _LL, _LL, _PLL, _LL, _PD, ctypes.c_double, ctypes.c_char_p]
    for name in ("remma_epiAA_maf_eff_cpu", "remma_epiDD_maf_eff_cpu"):
        getattr(epi, name).argtypes = [ctypes.c_char_p, _LL, _LL, _PLL, _LL, _PD, _PLL, _PD, ctypes.c_char_p]
    epi.remma_epiAD_maf_eff_cpu.argtypes = [ctypes.c_char_p, _LL, _LL, _PLL, _LL, _PD, _PLL, _PLL, _PD,
                                            ctypes.c_char_p]
    m_eff = types.ModuleType("_cremma_epi_eff_cpu")
    m_eff.ffi = _Ffi()
    m_eff.lib = _EffLib(epi)
    sys.modules["_cremma_epi_eff_cpu"] = m_eff

    rb = ctypes.CDLL(os.path.join(_REF_LIB, "libreadbed.so"))
    rb.read_plink_bed.argtypes = [ctypes.c_char_p, _LL, _LL, _PD]
    m_rb = types.ModuleType("_cread_plink_bed")
    m_rb.ffi = _Ffi()
    m_rb.lib = _EffLib(rb)
    sys.modules["_cread_plink_bed"] = m_rb

    # never load the .pyc files that ship inside the reference: keep bytecode in a private prefix
    sys.pycache_prefix = "/tmp/gmat_ref_pycache"
    sys.dont_write_bytecode = True
    # the repo ships its own `gmat` alias package (resolving to gmat_amd): drop any cached gmat*
    # modules and put the reference first, then make sure the reference's package is what loaded
    for name in [k for k in sys.modules if k == "gmat" or k.startswith("gmat.")]:
        del sys.modules[name]
    while REF_ROOT in sys.path:
        sys.path.remove(REF_ROOT)
    sys.path.insert(0, REF_ROOT)
    import gmat  # noqa: F401
    got = os.path.realpath(gmat.__file__)
    if not got.startswith(os.path.realpath(REF_ROOT) + os.sep):
        raise ImportError("import_reference: `gmat` resolved to %s, not the reference under %s" % (got, REF_ROOT))
    return gmat
