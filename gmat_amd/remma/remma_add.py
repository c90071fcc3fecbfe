"""Single-SNP additive test by random SNP-BLUP -- drop-in for gmat.remma.remma_add
(remma_add.py:15-77).  P and Z'Py come from the device projection; the per-SNP products
x'Py and x'Px (the reference's np.dot(snp_mat.T, pymat) and the n x n x m product at :58-59)
run on the GPU (gmat_snp_test); scaling, the chi2 test and the output table follow the
reference's expressions and writer."""
import logging

import numpy as np
import pandas as pd
from scipy.stats import chi2

from .. import _native as N
from .. import dist
from ..plink import Geno
from ..uvlmm.design_matrix import design_matrix_wemai_multi_gmat
from ..uvlmm.uvlmm_varcom import projection


def snp_products(bed_file, pvp, py, kind):
    """(x'Py, x'Px, scale) for every SNP of the imputed panel (kind GMAT_GRM_ADD / _DOM)."""
    with Geno(bed_file) as geno:
        if geno.n != pvp.shape[0]:
            raise ValueError("Z has %d individuals, the .fam has %d" % (pvp.shape[0], geno.n))
        xpy = np.zeros(geno.m)
        xpx = np.zeros(geno.m)
        N.check(N.load().gmat_snp_test(geno.handle, kind, N.ptr(N.f64(pvp)), N.ptr(N.f64(py)), N.ptr(xpy),
                                       N.ptr(xpx)), "gmat_snp_test")
        freq = geno.freq()
    if kind == N.GMAT_GRM_ADD:
        scale = np.sum(2 * freq * (1 - freq))
    else:
        scale_vec = 2 * freq * (1 - freq)
        scale = np.sum(scale_vec * (1 - scale_vec))
    return xpy, xpx, scale


def single_snp_table(bed_file, xpy, xpx, scale, sigma):
    """The reference's statistics (remma_add.py:58-75) and result table."""
    with np.errstate(divide="ignore", invalid="ignore"):
        eff_vec = xpy * sigma / scale
        var_vec = xpx * sigma * sigma / (scale * scale)
        eff_vec_to_fixed = eff_vec * sigma / (var_vec * scale)
        chi_vec = eff_vec * eff_vec / var_vec
    p_vec = chi2.sf(chi_vec, 1)
    snp_info = pd.read_csv(bed_file + ".bim", sep=r"\s+", header=None)
    res_df = snp_info.iloc[:, [0, 1, 3, 4, 5]].copy()
    res_df.columns = ["chro", "snp_ID", "pos", "allele1", "allele2"]
    res_df.loc[:, "eff_val"] = eff_vec
    res_df.loc[:, "chi_val"] = chi_vec
    res_df.loc[:, "eff_val_to_fixed"] = eff_vec_to_fixed
    res_df.loc[:, "p_val"] = p_vec
    return res_df


@dist.on_root
def _remma_add(y, xmat, zmat, gmat_lst, var_com, bed_file, out_file='remma_add'):
    """Writes out_file ('chro snp_ID pos allele1 allele2 eff_val chi_val eff_val_to_fixed p_val')
    and returns the DataFrame.  var_com[0] is the additive variance."""
    logging.info("Calculate the phenotypic covariance matrix and inversion")
    pvp, py = projection(y, xmat, zmat, gmat_lst, var_com)
    xpy, xpx, scale = snp_products(bed_file, pvp, py, N.GMAT_GRM_ADD)
    logging.info("Scaled factors {:.3f}".format(scale))
    res_df = single_snp_table(bed_file, xpy, xpx, scale, var_com[0])
    res_df.to_csv(out_file, index=False, header=True, sep=' ')
    return res_df


def remma_add(pheno_file, bed_file, gmat_lst, var_com, out_file='remma_add'):
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    return _remma_add(y, xmat, zmat, gmat_lst, var_com, bed_file, out_file=out_file)


