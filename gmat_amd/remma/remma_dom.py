"""Single-SNP dominance test by random SNP-BLUP -- drop-in for gmat.remma.remma_dom
(remma_dom.py:15-79): the dominance coding [g != 2] g - 2p(1-p), scale sum(s(1-s)) with
s = 2p(1-p), and var_com[1] as the dominance variance.  Device work as in remma_add."""
import logging

from .. import _native as N
from .. import dist
from ..uvlmm.design_matrix import design_matrix_wemai_multi_gmat
from ..uvlmm.uvlmm_varcom import projection
from .remma_add import single_snp_table, snp_products


@dist.on_root
def _remma_dom(y, xmat, zmat, gmat_lst, var_com, bed_file, out_file='remma_dom'):
    logging.info("Calculate the phenotypic covariance matrix and inversion")
    pvp, py = projection(y, xmat, zmat, gmat_lst, var_com)
    xpy, xpx, scale = snp_products(bed_file, pvp, py, N.GMAT_GRM_DOM)
    logging.info('The scaled factor is: {:.3f}'.format(scale))
    res_df = single_snp_table(bed_file, xpy, xpx, scale, var_com[1])
    res_df.to_csv(out_file, index=False, header=True, sep=' ')
    return res_df


def remma_dom(pheno_file, bed_file, gmat_lst, var_com, out_file='remma_dom'):
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    return _remma_dom(y, xmat, zmat, gmat_lst, var_com, bed_file, out_file=out_file)
