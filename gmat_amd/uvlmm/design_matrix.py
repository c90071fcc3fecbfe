"""Phenotype / design matrices -- drop-in for gmat.uvlmm.design_matrix (host-side parsing)."""
import logging

import numpy as np
from scipy.sparse import csr_matrix

_NA = ("NA", "NaN", "nan", "na")


def design_matrix_wemai_multi_gmat(pheno_file, bed_file):
    """y, X and the record->individual incidence Z (csr), in .fam order
    (design_matrix.py:7-57).  A genotyped id without a phenotype raises ValueError
    (the reference logs it and calls sys.exit(), :31-34)."""
    fam = []
    with open(bed_file + ".fam") as f:
        for line in f:
            a = line.split()
            fam.append(a[0] + " " + a[1])
    recs = {}
    with open(pheno_file) as f:
        for line in f:
            a = line.split()
            if a[-1] in _NA:
                continue
            recs.setdefault(a[0] + " " + a[1], []).append(a)
    missing = set(fam) - set(recs)
    if missing:
        msg = "The below genotyped id is not in the phenotype file:\n {}".format("\n".join(sorted(missing)))
        logging.error(msg)
        raise ValueError(msg)
    y, x, iid = [], [], []
    for key in fam:
        for a in recs[key]:
            y.append(float(a[-1]))
            x.append(a[2:-1])
            iid.append(a[1])
    y = np.array(y).reshape(-1, 1)
    xmat = np.array(x, dtype=float).reshape(y.shape[0], -1)
    order, col = {}, []
    for v in iid:
        if v not in order:
            order[v] = len(order)
        col.append(order[v])
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
    fam = []
    with open(bed_file + ".fam") as f:
        for line in f:
            a = line.split()
            fam.append(a[0] + " " + a[1])
    recs = {}
    with open(pheno_file) as f:
        for line in f:
            a = line.split()
            if a[-1] in _NA:
                continue
            recs.setdefault(a[0] + " " + a[1], []).append(a)
    y, x, iid = [], [], []
    for key in fam:
        if key in recs:
            for a in recs[key]:
                y.append(float(a[-1]))
                x.append(a[2:-1])
                iid.append(a[1])
        else:
            iid.append(None)
    y = np.array(y).reshape(-1, 1)
    xmat = np.array(x, dtype=float).reshape(y.shape[0], -1)
    order, rows, col = {}, 0, []
    n_col = 0
    for v in iid:
        if v is None:
            n_col += 1
            continue
        if v not in order:
            order[v] = n_col
            n_col += 1
        col.append(order[v])
        rows += 1
    zmat = csr_matrix((np.ones(rows), (np.arange(rows), col)), shape=(rows, n_col))
    return y, xmat, zmat
