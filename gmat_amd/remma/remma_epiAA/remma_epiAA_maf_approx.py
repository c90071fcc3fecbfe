"""Approximate additive by additive test with frequency-class variance denominators -- drop-in for
gmat.remma.remma_epiAA.remma_epiAA_maf_approx (remma_epiAA_maf_approx.py).  ``seed`` as in
remma_epiAA_approx."""
from .._eff import run_maf_approx


def remma_epiAA_maf_approx(pheno_file, bed_file, gmat_lst, var_com, p_cut=1.0e-5, num_random_pair=100000,
                           out_file='epiAA_maf_approx', seed=None):
    return run_maf_approx("AA", pheno_file, bed_file, gmat_lst, var_com, p_cut=p_cut,
                          num_random_pair=num_random_pair, out_file=out_file, seed=seed)


def remma_epiAA_maf_approx_parallel(pheno_file, bed_file, gmat_lst, var_com, parallel, p_cut=1.0e-5,
                                    num_random_pair=100000, out_file='epiAA_maf_approx_parallel', seed=None):
    return run_maf_approx("AA", pheno_file, bed_file, gmat_lst, var_com, p_cut=p_cut,
                          num_random_pair=num_random_pair, out_file=out_file, parallel=parallel, seed=seed)
