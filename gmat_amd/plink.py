"""PLINK binary fileset input and the device-resident genotype panel.

``read_plink`` (process_plink.py:7-9) in the reference decodes the whole .bed into an
n x m float matrix through pandas_plink.  Here the packed 2-bit .bed body goes to the GPU
as is (25 MB for 2,000 x 50,000) and is decoded there (gmat_geno_create); the host only
validates the file and, when calls are missing, imputes them the way impute_geno
(process_plink.py:12-25) does before upload.
"""
import ctypes

import numpy as np

from . import _native as N

BED_MAGIC = b"\x6c\x1b\x01"


def count_lines(path):
    """Lines as iterating the file counts them (a last line without a newline included): newlines
    counted in 1-MiB blocks (~10x faster than the line iteration on a 50,000-SNP .bim)."""
    n, last = 0, b"\n"
    with open(path, "rb") as f:
        while True:
            blk = f.read(1 << 20)
            if not blk:
                break
            n += blk.count(b"\n")
            last = blk[-1:]
    return n + (last != b"\n")


def read_fam_ids(bed_file):
    fid, iid = [], []
    with open(bed_file + ".fam") as f:
        for line in f:
            a = line.split()
            fid.append(a[0])
            iid.append(a[1])
    return fid, iid


def read_bed_body(bed_file):
    """Return (body uint8 array, n_id, n_snp) with the magic and size checked."""
    n = count_lines(bed_file + ".fam")
    m = count_lines(bed_file + ".bim")
    with open(bed_file + ".bed", "rb") as f:
        raw = f.read()
    if raw[:3] != BED_MAGIC:
        raise ValueError("%s.bed is not a SNP-major PLINK .bed (magic %r)" % (bed_file, raw[:3]))
    nb = (n + 3) // 4
    body = np.frombuffer(raw, dtype=np.uint8, offset=3)
    if body.size < nb * m:
        raise ValueError("%s.bed has %d data bytes; %d SNPs x %d individuals need %d"
                         % (bed_file, body.size, m, n, nb * m))
    return body[: nb * m], n, m


def _codes(body, n, m):
    nb = (n + 3) // 4
    raw = body.reshape(m, nb)
    return np.stack([(raw >> (2 * k)) & 3 for k in range(4)], axis=-1).reshape(m, nb * 4)[:, :n]


def _pack(codes):
    m, n = codes.shape
    nb = (n + 3) // 4
    pad = np.zeros((m, nb * 4), dtype=np.uint8)
    pad[:, :n] = codes
    pad = pad.reshape(m, nb, 4)
    return (pad[:, :, 0] | (pad[:, :, 1] << 2) | (pad[:, :, 2] << 4) | (pad[:, :, 3] << 6)).astype(np.uint8).ravel()


def missing_column_order(miss_nm):
    """SNP columns holding missing calls, in the order impute_geno visits them: the
    iteration order of ``set(np.where(np.isnan(snp_mat))[1])`` on the n x m matrix
    (process_plink.py:13-15).  With the same np.random state the draws are then the
    reference's own."""
    return list(set(np.where(miss_nm)[1]))


def impute_missing(body, n, m, rng=None):
    """Replace missing calls (code 01) per SNP by random draws from that SNP's observed
    0/1/2 frequencies, as impute_geno (process_plink.py:12-25): same column order, same
    probabilities (count / total as float64) and the same np.random.choice call, so a
    caller that seeds np.random gets the reference's imputed genotypes.  The reference's
    draws are unseeded, so imputed genotypes are not reproducible there by default."""
    rng = np.random if rng is None else rng
    codes = _codes(body, n, m)
    miss = codes == 1
    if not miss.any():
        return body
    codes = codes.copy()
    dose_code = np.array([0b00, 0b10, 0b11], dtype=np.uint8)
    for j in missing_column_order(miss.T):
        c = codes[j]
        cnt = [np.sum(c == 0), np.sum(c == 2), np.sum(c == 3)]
        tot = cnt[0] + cnt[1] + cnt[2]
        k = miss[j]
        draw = rng.choice([0.0, 1.0, 2.0], int(k.sum()), p=[cnt[0] / tot, cnt[1] / tot, cnt[2] / tot])
        c[k] = dose_code[draw.astype(np.int64)]
    return _pack(codes)


class Geno:
    """Device-resident genotype panel (gmat_geno handle)."""

    def __init__(self, bed_file=None, body=None, n_id=None, n_snp=None, impute=True):
        lib = N.ensure_device()
        if bed_file is not None:
            body, n_id, n_snp = read_bed_body(bed_file)
        self.n, self.m = int(n_id), int(n_snp)
        body = np.ascontiguousarray(body, dtype=np.uint8)
        h = ctypes.c_void_p()
        N.check(lib.gmat_geno_create(ctypes.byref(h), N.ptr(body), body.size, self.n, self.m), "gmat_geno_create")
        self._h = h
        self._lib = lib
        self.sum_dose, self.n_het, self.n_miss = self.counts()
        if impute and self.n_miss.sum() > 0:
            self.close()
            body = impute_missing(body, self.n, self.m)
            h = ctypes.c_void_p()
            N.check(lib.gmat_geno_create(ctypes.byref(h), N.ptr(body), body.size, self.n, self.m),
                    "gmat_geno_create")
            self._h = h
            self.sum_dose, self.n_het, self.n_miss = self.counts()

    @property
    def handle(self):
        return self._h

    def counts(self):
        s = np.zeros(self.m, np.int64)
        h = np.zeros(self.m, np.int64)
        mi = np.zeros(self.m, np.int64)
        N.check(self._lib.gmat_geno_counts(self._h, N.ptr(s), N.ptr(h), N.ptr(mi)), "gmat_geno_counts")
        return s, h, mi

    def freq(self):
        """Allele frequency of the counted allele, computed as the reference does
        (np.sum(snp_mat, axis=0) / (2 * num_id))."""
        return self.sum_dose / (2 * self.n)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.gmat_geno_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
