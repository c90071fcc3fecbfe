"""Exact AA epistasis scan on the GPU -- drop-in for gmat.remma.remma_epiAA (remma_epiAA.py:16-161)."""
from ...uvlmm.design_matrix import design_matrix_wemai_multi_gmat
from .._scan import run_parallel, run_scan


def _remma_epiAA(y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=None, p_cut=1.0e-5, out_file='epiAA'):
    """Writes out_file: 'snp_0 snp_1 eff chi p_val' + the pairs with p < p_cut; returns 0."""
    return run_scan("AA", y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0, p_cut, out_file)


def remma_epiAA(pheno_file, bed_file, gmat_lst, var_com, snp_lst_0=None, p_cut=1.0e-5, out_file='epiAA'):
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    return _remma_epiAA(y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=snp_lst_0, p_cut=p_cut,
                         out_file=out_file)


def _remma_epiAA_parallel(y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, p_cut=1.0e-5,
                           out_file='epiAA_parallel'):
    """Part parallel[1] of parallel[0] (triangle-folded rows); writes out_file + '.k'."""
    return run_parallel("AA", y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, p_cut, out_file)


def remma_epiAA_parallel(pheno_file, bed_file, gmat_lst, var_com, parallel, p_cut=1.0e-5,
                          out_file='epiAA_parallel'):
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    return _remma_epiAA_parallel(y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, p_cut=p_cut,
                                  out_file=out_file)
