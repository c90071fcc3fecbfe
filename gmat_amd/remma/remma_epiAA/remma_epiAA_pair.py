"""AA epistasis test of a SNP-pair list on the GPU -- drop-in for
gmat.remma.remma_epiAA.remma_epiAA_pair (remma_epiAA_pair.py)."""
from ...uvlmm.design_matrix import design_matrix_wemai_multi_gmat
from .._scan import run_pairs


def _remma_epiAA_pair(y, xmat, zmat, gmat_lst, var_com, bed_file, snp_pair_file, max_test_pair=50000,
                       p_cut=1.0e-4, out_file='epiAA_pair'):
    """Writes out_file: 'snp_0 snp_1 eff var chi p' + the listed pairs with p < p_cut."""
    return run_pairs("AA", y, xmat, zmat, gmat_lst, var_com, bed_file, snp_pair_file, max_test_pair, p_cut,
                     out_file)


def remma_epiAA_pair(pheno_file, bed_file, gmat_lst, var_com, snp_pair_file, max_test_pair=50000, p_cut=1.0e-4,
                      out_file='epiAA_pair'):
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    return _remma_epiAA_pair(y, xmat, zmat, gmat_lst, var_com, bed_file, snp_pair_file,
                              max_test_pair=max_test_pair, p_cut=p_cut, out_file=out_file)
