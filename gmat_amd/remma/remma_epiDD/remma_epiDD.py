"""Exact DD epistasis scan on the GPU -- drop-in for gmat.remma.remma_epiDD (remma_epiDD.py:16-165)."""
from ...uvlmm.design_matrix import design_matrix_wemai_multi_gmat
from .._scan import run_parallel, run_scan


def _remma_epiDD(y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=None, p_cut=0.0001, out_file='epiDD'):
    """Writes out_file: 'snp_0 snp_1 eff chi p_val' + the pairs with p < p_cut; returns 0."""
    return run_scan("DD", y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0, p_cut, out_file)


def remma_epiDD(pheno_file, bed_file, gmat_lst, var_com, snp_lst_0=None, p_cut=1.0e-5, out_file='epiDD'):
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    return _remma_epiDD(y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=snp_lst_0, p_cut=p_cut,
                         out_file=out_file)


def _remma_epiDD_parallel(y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, p_cut=1.0e-4,
                           out_file='epiDD_parallel'):
    """Part parallel[1] of parallel[0] (triangle-folded rows); writes out_file + '.k'."""
    return run_parallel("DD", y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, p_cut, out_file)


def remma_epiDD_parallel(pheno_file, bed_file, gmat_lst, var_com, parallel, p_cut=1.0e-5,
                          out_file='epiDD_parallel'):
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    return _remma_epiDD_parallel(y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, p_cut=p_cut,
                                  out_file=out_file)
