"""Effect-only additive by additive screen -- drop-in for gmat.remma.remma_epiAA.remma_epiAA_eff
(remma_epiAA_eff.py).  The screen runs on the GPU behind the reference's C symbol
remma_epiAA_eff_cpu (include/gmat_remma_eff.h); host logic in .._eff."""
from ...uvlmm.design_matrix import design_matrix_wemai_multi_gmat
from .._eff import run_eff, run_eff_parallel


def _remma_epiAA_eff(y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=None, var_app=1.0, p_cut=1.0e-5,
                     out_file='epiAA_eff'):
    """Writes out_file: 'snp_0 snp_1 eff chi_app p_app' for |eff| above sqrt(chi2.isf(p_cut, 1) * var_app)."""
    return run_eff("AA", y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=snp_lst_0, var_app=var_app,
                   p_cut=p_cut, out_file=out_file)


def remma_epiAA_eff(pheno_file, bed_file, gmat_lst, var_com, snp_lst_0=None, var_app=1.0, p_cut=1.0e-5,
                    out_file='epiAA_eff'):
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    return _remma_epiAA_eff(y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=snp_lst_0, var_app=var_app,
                            p_cut=p_cut, out_file=out_file)


def _remma_epiAA_eff_parallel(y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, var_app=1.0, p_cut=1.0e-5,
                              out_file='epiAA_eff_parallel'):
    """Part parallel[1] of parallel[0] (triangle-folded rows); writes out_file + '.k'."""
    return run_eff_parallel("AA", y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, var_app=var_app,
                            p_cut=p_cut, out_file=out_file)


def remma_epiAA_eff_parallel(pheno_file, bed_file, gmat_lst, var_com, parallel, var_app=1.0, p_cut=1.0e-5,
                             out_file='epiAA_eff_parallel'):
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    return _remma_epiAA_eff_parallel(y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, var_app=var_app,
                                     p_cut=p_cut, out_file=out_file)
