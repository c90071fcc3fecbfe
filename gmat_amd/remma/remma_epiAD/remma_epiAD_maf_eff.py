"""Effect-only additive by dominance screen with frequency-class thresholds -- drop-in for
gmat.remma.remma_epiAD.remma_epiAD_maf_eff (remma_epiAD_maf_eff.py).  The screen runs on the GPU
behind remma_epiAD_maf_eff_cpu (include/gmat_remma_eff.h); host logic in .._eff.
Default output names are the reference's."""
from ...uvlmm.design_matrix import design_matrix_wemai_multi_gmat
from .._eff import run_maf_eff, run_maf_eff_parallel


def _remma_epiAD_maf_eff(y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=None, freqA=None, freqD=None, freq_deno=None,
                         p_cut=1.0e-5, out_file='epiAD_maf_eff'):
    return run_maf_eff("AD", y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=snp_lst_0, freq_i=freqA, freq_j=freqD,
                       freq_deno=freq_deno, p_cut=p_cut, out_file=out_file)


def remma_epiAD_maf_eff(pheno_file, bed_file, gmat_lst, var_com, snp_lst_0=None, freqA=None, freqD=None, freq_deno=None,
                        p_cut=1.0e-5, out_file='epiAA_maf_eff'):
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    return _remma_epiAD_maf_eff(y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=snp_lst_0, freqA=freqA, freqD=freqD,
                                freq_deno=freq_deno, p_cut=p_cut, out_file=out_file)


def _remma_epiAD_maf_eff_parallel(y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, freqA=None, freqD=None, freq_deno=None,
                                  p_cut=1.0e-5, out_file='epiAA_maf_eff_parallel'):
    return run_maf_eff_parallel("AD", y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, freq_i=freqA, freq_j=freqD,
                                freq_deno=freq_deno, p_cut=p_cut, out_file=out_file)


def remma_epiAD_maf_eff_parallel(pheno_file, bed_file, gmat_lst, var_com, parallel, freqA=None, freqD=None, freq_deno=None,
                                 p_cut=1.0e-5, out_file='epiAA_maf_eff_parallel'):
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    return _remma_epiAD_maf_eff_parallel(y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, freqA=freqA, freqD=freqD,
                                         freq_deno=freq_deno, p_cut=p_cut, out_file=out_file)
