"""Approximate additive by additive test -- drop-in for gmat.remma.remma_epiAA.remma_epiAA_approx
(remma_epiAA_approx.py): random pairs -> median exact variance -> GPU effect screen ->
exact re-test of the survivors -> 'snp_0 snp_1 eff var chi p_app p'.  ``seed`` (an addition,
default None = unseeded like the reference) makes the random pairs reproducible."""
from .._eff import run_approx


def remma_epiAA_approx(pheno_file, bed_file, gmat_lst, var_com, p_cut=1.0e-5, num_random_pair=100000,
                       out_file='epiAA_approx', seed=None):
    return run_approx("AA", pheno_file, bed_file, gmat_lst, var_com, p_cut=p_cut, num_random_pair=num_random_pair,
                      out_file=out_file, seed=seed)


def remma_epiAA_approx_parallel(pheno_file, bed_file, gmat_lst, var_com, parallel, p_cut=1.0e-5,
                                num_random_pair=100000, out_file='epiAA_approx', seed=None):
    return run_approx("AA", pheno_file, bed_file, gmat_lst, var_com, p_cut=p_cut, num_random_pair=num_random_pair,
                      out_file=out_file, parallel=parallel, seed=seed)
