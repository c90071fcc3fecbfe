"""Weighted EM-AI REML on the GPU -- drop-in for gmat.uvlmm.uvlmm_varcom.

The iteration of _wemai_multi_gmat (uvlmm_varcom.py:8-104) runs in libgmat_hip
(gmat_amd/csrc/reml.hip): Cholesky of V, V^-1, P, the traces and the AI matrix on the
device; the (c+1)-sized weight search and the convergence test on the host.
"""
import ctypes
import logging

import numpy as np

from .. import _native as N
from .. import dist
from .design_matrix import design_matrix_wemai_multi_gmat, design_matrix_wemai_multi_gmat_pred, z_columns


def _gmat_ptrs(gmat_lst, n_id):
    mats = [N.f64(g) for g in gmat_lst]
    for g in mats:
        if g.shape != (n_id, n_id):
            raise ValueError("relationship matrix of shape %s, expected %s" % (g.shape, (n_id, n_id)))
    arr = (ctypes.c_void_p * max(1, len(mats)))(*[g.ctypes.data for g in mats])
    return mats, arr


@dist.on_root
def _wemai_multi_gmat(y, xmat, zmat, gmat_lst, init=None, maxiter=200, cc_par=1.0e-8, cc_gra=1.0e-6):
    """Estimate the variance components (residual last).  Same arguments and result as
    uvlmm_varcom.py:8."""
    lib = N.ensure_device()
    y = N.f64(np.asarray(y).reshape(-1))
    n = y.shape[0]
    xmat = N.f64(np.asarray(xmat).reshape(n, -1))
    col, n_id = z_columns(zmat, n)
    mats, arr = _gmat_ptrs(gmat_lst, n_id)
    c1 = len(mats) + 1
    init_arr = None if init is None else N.f64(np.asarray(init, dtype=float).reshape(-1))
    if init_arr is not None and init_arr.size != c1:
        raise ValueError("init must have %d values" % c1)
    var = np.zeros(c1)
    hist = np.zeros((max(1, maxiter), c1))
    it = ctypes.c_int(0)
    logging.info("Initial variances: " + " ".join(map(str, init_arr if init_arr is not None else [1.0] * c1)))
    N.check(lib.gmat_reml(n, xmat.shape[1], n_id, len(mats), N.ptr(y), N.ptr(xmat), N.ptr(col), arr,
                          N.ptr(init_arr), int(maxiter), float(cc_par), float(cc_gra), N.ptr(var),
                          ctypes.byref(it), N.ptr(hist)), "gmat_reml")
    for k in range(it.value):
        logging.info("Updated variances: " + " ".join(map(str, hist[k])))
    _wemai_multi_gmat.last_history = hist[: it.value].copy()
    tr = np.zeros((3, max(1, it.value)))
    cnt = ctypes.c_int(0)
    N.check(lib.gmat_reml_trace(tr.shape[1], N.ptr(tr[0]), N.ptr(tr[1]), N.ptr(tr[2]), ctypes.byref(cnt)),
            "gmat_reml_trace")
    # per iteration: norm of the gradient vector, norm of the update vector, EM weight (uvlmm_varcom.py:90-96)
    _wemai_multi_gmat.last_trace = tr[:, : it.value].copy()
    return var


@dist.on_root
def wemai_multi_gmat(pheno_file, bed_file, gmat_lst, init=None, maxiter=200, cc_par=1.0e-8, cc_gra=1.0e-6,
                     out_file="wemai_multi_gmat.var"):
    """uvlmm_varcom.py:107-126: design matrices, REML, np.savetxt(out_file, var_com)."""
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    var_com = _wemai_multi_gmat(y, xmat, zmat, gmat_lst, init=init, maxiter=maxiter, cc_par=cc_par, cc_gra=cc_gra)
    np.savetxt(out_file, var_com)
    return var_com


@dist.on_root
def predict_random(y, xmat, zmat, gmat_lst, var_com):
    """rand_eff (n_id x len(gmat_lst)) of wemai_multi_gmat_pred (uvlmm_varcom.py:147-165), on the
    device (gmat_blup), with the reference's formula as written there."""
    lib = N.ensure_device()
    y = N.f64(np.asarray(y).reshape(-1))
    n = y.shape[0]
    xmat = N.f64(np.asarray(xmat).reshape(n, -1))
    col, n_id = z_columns(zmat, n)
    mats, arr = _gmat_ptrs(gmat_lst, n_id)
    var = N.f64(np.asarray(var_com, dtype=float).reshape(-1))
    if var.size != len(mats) + 1:
        raise ValueError("var_com must have %d values" % (len(mats) + 1))
    out = np.zeros((n_id, len(mats)))
    N.check(lib.gmat_blup(n, xmat.shape[1], n_id, len(mats), N.ptr(y), N.ptr(xmat), N.ptr(col), arr, N.ptr(var),
                          N.ptr(out)), "gmat_blup")
    return out


@dist.on_root
def wemai_multi_gmat_pred(pheno_file, bed_file, gmat_lst, init=None, maxiter=200, cc_par=1.0e-8, cc_gra=1.0e-6,
                          out_file='wemai_multi_gmat_pred'):
    """uvlmm_varcom.py:129-167: REML with genotyped-but-unphenotyped ids kept in Z, then the
    random-effect prediction; writes out_file + '.var' and out_file + '.rand_eff'."""
    y, xmat, zmat = design_matrix_wemai_multi_gmat_pred(pheno_file, bed_file)
    var_com = _wemai_multi_gmat(y, xmat, zmat, gmat_lst, init=init, maxiter=maxiter, cc_par=cc_par, cc_gra=cc_gra)
    np.savetxt(out_file + '.var', var_com)
    logging.info('Predict the random effects')
    rand_eff = predict_random(y, xmat, zmat, gmat_lst, var_com)
    np.savetxt(out_file + '.rand_eff', rand_eff)
    return var_com


@dist.on_root
def projection(y, xmat, zmat, gmat_lst, var_com):
    """(Z'PZ, Z'Py) of the scans' setup (remma_epiAA.py:33-49), computed on the device."""
    lib = N.ensure_device()
    y = N.f64(np.asarray(y).reshape(-1))
    n = y.shape[0]
    xmat = N.f64(np.asarray(xmat).reshape(n, -1))
    col, n_id = z_columns(zmat, n)
    mats, arr = _gmat_ptrs(gmat_lst, n_id)
    var = N.f64(np.asarray(var_com, dtype=float).reshape(-1))
    if var.size != len(mats) + 1:
        raise ValueError("var_com must have %d values" % (len(mats) + 1))
    pvp = np.empty((n_id, n_id))
    py = np.empty(n_id)
    N.check(lib.gmat_projection(n, xmat.shape[1], n_id, len(mats), N.ptr(y), N.ptr(xmat), N.ptr(col), arr,
                                N.ptr(var), N.ptr(pvp), N.ptr(py)), "gmat_projection")
    return pvp, py
