"""read_plink / impute_geno -- drop-in for gmat.process_plink.process_plink (process_plink.py:7-25).

``read_plink`` decodes the packed .bed on the device (gmat_geno_decode) and returns the
reference's n x m dosage matrix with NaN for missing calls (read_plink_bed.py:23-28).
``impute_geno`` fills the NaNs exactly as the reference does (host numpy; the draws use the
global np.random state in the reference's column order).
"""
import numpy as np

from .. import _native as N
from ..plink import Geno, missing_column_order


def read_plink(bed_file):
    """n x m float64 dosage (0/1/2, NaN = missing), individuals in .fam order."""
    with Geno(bed_file, impute=False) as g:
        mat = np.empty((g.m, g.n))
        N.check(N.load().gmat_geno_decode(g.handle, N.ptr(mat)), "gmat_geno_decode")
    mat[np.abs(mat - 1.0 / 3) < 0.0001] = np.nan
    return np.ascontiguousarray(mat.T)


def impute_geno(snp_mat):
    """In place: each NaN becomes a draw from its SNP's observed 0/1/2 frequencies
    (process_plink.py:12-25); returns snp_mat."""
    for i in missing_column_order(np.isnan(snp_mat)):
        snpi = snp_mat[:, i]
        cnt = [np.sum(np.absolute(snpi - v) < 1e-10) for v in (0.0, 1.0, 2.0)]
        tot = cnt[0] + cnt[1] + cnt[2]
        na = np.where(np.isnan(snpi))
        snpi[na] = np.random.choice([0.0, 1.0, 2.0], len(na[0]), p=[cnt[0] / tot, cnt[1] / tot, cnt[2] / tot])
        snp_mat[:, i] = snpi
    return snp_mat
