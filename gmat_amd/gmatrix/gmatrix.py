"""Genomic relationship matrices on the GPU -- drop-in for gmat.gmatrix (gmatrix.py).

``agmat`` / ``dgmat_as`` keep the reference signatures, outputs and files; the n x n
product runs as an exact int8 MFMA GEMM of the 0/1/2 codes with fp64 centring
corrections (gmat_amd/csrc/geno.hip), the optional inverse as a device Cholesky inverse.
"""
import ctypes
import logging
import time

import numpy as np

from .. import _native as N
from .. import dist
from ..plink import Geno, read_fam_ids


def _fam_ids_as_pandas(bed_file):
    """IDs as ``pd.read_csv(fam, sep='\\s+', header=None).iloc[:, 1]`` renders them
    (all-integer columns become ints)."""
    _, iid = read_fam_ids(bed_file)
    try:
        return np.array([int(v) for v in iid], dtype=np.int64)
    except ValueError:
        return np.array(iid, dtype=object)


@dist.on_root
def output_mat(mat, id, out_file, out_fmt):
    """Output of gmatrix.py:10-31: 'mat' (np.savetxt '%.18e', suffix 0), 'row_col_val' (1-based
    lower triangle, suffix 1), 'id_id_val' (suffix 2), byte-identical to the reference's
    writers but formatted by the library's multi-threaded C++ writer (gmat_write_grm_text).
    Addition: 'npy' writes the binary float64 matrix to out_file + '0.npy' (np.load-able)."""
    mat = N.f64(mat)
    fmt = {"mat": 0, "row_col_val": 1, "id_id_val": 2}.get(out_fmt)
    if out_fmt == "npy":
        np.save(out_file + "0.npy", mat)
        return 1
    if fmt is None:
        return 0
    blob = b"".join(str(v).encode() + b"\0" for v in id) if fmt == 2 else None
    N.check(N.load().gmat_write_grm_text((out_file + str(fmt)).encode(), N.ptr(mat), mat.shape[0], fmt, blob, 0),
            "gmat_write_grm_text")
    return 1


def _grm(bed_file, kind, inv, small_val, out_fmt, suffix, inv_suffix):
    if out_fmt not in ("mat", "row_col_val", "id_id_val", "npy"):
        raise ValueError("Not Recognized output format: " + str(out_fmt))
    lib = N.ensure_device()
    with Geno(bed_file) as g:
        logging.info("There are {:d} individuals and {:d} SNPs.".format(g.n, g.m))
        kin = np.empty((g.n, g.n), dtype=np.float64)
        scale = ctypes.c_double()
        t0 = time.perf_counter()
        N.check(lib.gmat_grm(g.handle, kind, float(small_val), N.ptr(kin), ctypes.byref(scale)), "gmat_grm")
        logging.info("The scaled factor is: {:.3f}".format(scale.value))
        logging.info("Running time: Clock time, {:.5f} sec.".format(time.perf_counter() - t0))
    ids = _fam_ids_as_pandas(bed_file)
    output_mat(kin, ids, bed_file + suffix, out_fmt)
    kin_inv = None
    if inv:
        kin_inv = spd_inverse(kin)
        output_mat(kin_inv, ids, bed_file + inv_suffix, out_fmt)
    return kin, kin_inv


@dist.on_root
def spd_inverse(a):
    """Inverse of a symmetric positive-definite matrix on the device (Cholesky)."""
    lib = N.ensure_device()
    a = N.f64(a)
    out = np.empty_like(a)
    ld = ctypes.c_double()
    N.check(lib.gmat_spd_inverse(a.shape[0], N.ptr(a), N.ptr(out), ctypes.byref(ld)), "gmat_spd_inverse")
    return out


@dist.on_root
def agmat(bed_file, inv=False, small_val=0.001, out_fmt="mat"):
    """Additive genomic relationship matrix (gmatrix.py:34-94).  Writes
    ``bed_file + '.agrm{0,1,2}'`` (and ``.agiv*`` when inv) and returns (kin, kin_inv)."""
    return _grm(bed_file, N.GMAT_GRM_ADD, inv, small_val, out_fmt, ".agrm", ".agiv")


@dist.on_root
def dgmat_as(bed_file, inv=False, small_val=0.001, out_fmt="mat"):
    """Dominance genomic relationship matrix (gmatrix.py:97-159).  Writes
    ``bed_file + '.dgrm_as*'`` (and ``.dgiv_as*``) and returns (kin, kin_inv)."""
    return _grm(bed_file, N.GMAT_GRM_DOM, inv, small_val, out_fmt, ".dgrm_as", ".dgiv_as")
