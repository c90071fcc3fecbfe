"""Phenotype / design matrices -- drop-in for gmat.uvlmm.design_matrix (host-side parsing)."""
import logging

import numpy as np
from scipy.sparse import csr_matrix

_NA = ("NA", "NaN", "nan", "na")


def _fam_keys(bed_file):
    """'FID IID' of every genotyped individual, in .fam order."""
    with open(bed_file + ".fam") as f:
        return [" ".join(line.split()[:2]) for line in f]


def _records(pheno_file):
    """Phenotype records (split lines) by 'FID IID', missing phenotypes (NA) dropped."""
    recs = {}
    with open(pheno_file) as f:
        for line in f:
            a = line.split()
            if a[-1] in _NA:
                continue
            recs.setdefault(a[0] + " " + a[1], []).append(a)
    return recs


def _y_x(rows):
    """y (column) and the covariate columns of the records in `rows`."""
    y = np.array([float(a[-1]) for a in rows]).reshape(-1, 1)
    xmat = np.array([a[2:-1] for a in rows], dtype=float).reshape(y.shape[0], -1)
    return y, xmat


def design_matrix_wemai_multi_gmat(pheno_file, bed_file):
    """y, X and the record->individual incidence Z (csr), in .fam order
    (design_matrix.py:7-57).  A genotyped id without a phenotype raises ValueError
    (the reference logs it and calls sys.exit(), :31-34)."""
    fam, recs = _fam_keys(bed_file), _records(pheno_file)
    missing = set(fam) - set(recs)
    if missing:
        msg = "The below genotyped id is not in the phenotype file:\n {}".format("\n".join(sorted(missing)))
        logging.error(msg)
        raise ValueError(msg)
    rows = [a for key in fam for a in recs[key]]
    y, xmat = _y_x(rows)
    order, col = {}, []
    for a in rows:
        col.append(order.setdefault(a[1], len(order)))
    zmat = csr_matrix((np.ones(len(col)), (np.arange(len(col)), col)))
    return y, xmat, zmat


def z_columns(zmat, n_rec):
    """Record -> individual index of an incidence matrix (one 1.0 per row)."""
    z = csr_matrix(zmat)
    if z.shape[0] != n_rec:
        raise ValueError("Z has %d rows, expected %d" % (z.shape[0], n_rec))
    nnz = np.diff(z.indptr)
    if not (np.all(nnz == 1) and np.all(z.data == 1.0)):
        raise ValueError("Z must be an incidence matrix (exactly one 1.0 per record)")
    return np.ascontiguousarray(z.indices, dtype=np.int64), z.shape[1]


def design_matrix_wemai_multi_gmat_pred(pheno_file, bed_file):
    """As design_matrix_wemai_multi_gmat, but genotyped ids without a phenotype are allowed:
    they keep a (record-less) column of Z so that their random effects are predicted
    (design_matrix.py:60-113)."""
    fam, recs = _fam_keys(bed_file), _records(pheno_file)
    rows = [a for key in fam for a in recs.get(key, [])]
    y, xmat = _y_x(rows)
    order, col, n_col = {}, [], 0
    for key in fam:
        if key not in recs:  # a record-less id: its own column
            n_col += 1
            continue
        for a in recs[key]:
            if a[1] not in order:
                order[a[1]] = n_col
                n_col += 1
            col.append(order[a[1]])
    zmat = csr_matrix((np.ones(len(col)), (np.arange(len(col)), col)), shape=(len(col), n_col))
    return y, xmat, zmat
