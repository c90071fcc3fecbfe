"""Deterministic synthetic PLINK cohorts for tests and bench.py.

Individuals are *related* (a founder pool followed by generations of random mating with
block recombination), so that the A and A x A relationship matrices are distinguishable
from the identity and the REML is identifiable.  Genotypes are
written in SNP-major PLINK .bed order (magic 6c 1b 01, 2 bits per genotype, low bits
first, code 00 = hom first allele -> dosage 0, 10 = het -> 1, 11 = hom second allele -> 2,
01 = missing), i.e. the dosage convention of gmat/process_plink/_read_plink_bed.c:37.
"""
import os

import numpy as np

# dosage -> 2-bit PLINK code (counting the second .bim allele, as the reference decoder does)
_DOSE_TO_CODE = np.array([0b00, 0b10, 0b11], dtype=np.uint8)
MISSING_CODE = 0b01


def simulate_genotypes(n_id, n_snp, seed=1, n_founder=60, n_gen=6, block=250, maf_min=0.01, family_size=None):
    """Return an (n_snp, n_id) uint8 dosage matrix in {0,1,2} (SNP-major).  With family_size f the
    last generation comes in full-sib families of f (both parents shared), which makes A and A x A
    clearly distinct from the identity (the configs[1] REML cohort)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    freq = rng.uniform(0.1, 0.9, size=n_snp)
    n_blk = (n_snp + block - 1) // block
    # founder haplotypes: (2*n_founder, n_snp) bool
    pop = rng.random((2 * n_founder, n_snp)) < freq
    n_pop = n_founder
    for g in range(n_gen):
        n_next = n_id if g == n_gen - 1 else max(n_id, n_pop)
        new = np.empty((2 * n_next, n_snp), dtype=bool)
        fam = None
        if family_size and g == n_gen - 1:
            fam = rng.integers(0, n_pop, size=(2, (n_next + family_size - 1) // family_size))
        for side in range(2):
            par = rng.integers(0, n_pop, size=n_next) if fam is None else np.repeat(fam[side], family_size)[:n_next]
            pick = rng.integers(0, 2, size=(n_next, n_blk), dtype=np.uint8)
            pick = np.repeat(pick, block, axis=1)[:, :n_snp].astype(bool)
            h0 = pop[2 * par]
            h1 = pop[2 * par + 1]
            new[side::2] = np.where(pick, h1, h0)
        pop, n_pop = new, n_next
    geno = (pop[0::2].astype(np.uint8) + pop[1::2].astype(np.uint8)).T.copy()  # (n_snp, n_id)
    # forbid (near-)monomorphic SNPs: resample them independently at p=0.5
    p = geno.sum(axis=1) / (2.0 * n_id)
    bad = np.where(np.minimum(p, 1 - p) < maf_min)[0]
    if bad.size:
        geno[bad] = rng.binomial(2, 0.5, size=(bad.size, n_id)).astype(np.uint8)
    return geno


def simulate_genotype_shard(n_id, n_snp, lo, hi, seed=1, n_founder=60, n_gen=6, block=250, maf_min=0.01,
                            family_size=None):
    """SNPs [lo, hi) of ``simulate_genotypes(n_id, n_snp, seed)`` -- the same cohort, bit for bit --
    with only the shard's columns propagated through the pedigree (the expensive part); every
    random draw is made in the same order and size as the full generator (they are cheap), so
    each rank of a sharded run makes just its own SNP range.  Returns ((hi - lo, n_id) uint8,
    n_bad): n_bad counts this range's (near-)monomorphic SNPs, which the full generator re-draws
    at the end of its stream -- a caller whose ranks find any must fall back to the full
    generator (never the case for the bench cohorts)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    freq = rng.uniform(0.1, 0.9, size=n_snp)
    n_blk = (n_snp + block - 1) // block
    pop = (rng.random((2 * n_founder, n_snp)) < freq)[:, lo:hi]
    b_lo, b_hi = lo // block, (max(hi, lo + 1) - 1) // block + 1  # blocks the range touches
    n_pop = n_founder
    for g in range(n_gen):
        n_next = n_id if g == n_gen - 1 else max(n_id, n_pop)
        new = np.empty((2 * n_next, hi - lo), dtype=bool)
        fam = None
        if family_size and g == n_gen - 1:
            fam = rng.integers(0, n_pop, size=(2, (n_next + family_size - 1) // family_size))
        for side in range(2):
            par = rng.integers(0, n_pop, size=n_next) if fam is None else np.repeat(fam[side], family_size)[:n_next]
            pick = rng.integers(0, 2, size=(n_next, n_blk), dtype=np.uint8)
            pick = np.repeat(pick[:, b_lo:b_hi], block, axis=1)[:, lo - b_lo * block:hi - b_lo * block].astype(bool)
            new[side::2] = np.where(pick, pop[2 * par + 1], pop[2 * par])
        pop, n_pop = new, n_next
    geno = (pop[0::2].astype(np.uint8) + pop[1::2].astype(np.uint8)).T.copy()  # (hi - lo, n_id)
    p = geno.sum(axis=1) / (2.0 * n_id)
    n_bad = int(np.sum(np.minimum(p, 1 - p) < maf_min))
    return geno, n_bad


def pack_bed(geno, missing=None):
    """Pack an (n_snp, n_id) dosage matrix into PLINK .bed bytes (with the 3-byte magic)."""
    m, n = geno.shape
    nb = (n + 3) // 4
    codes = _DOSE_TO_CODE[geno]
    if missing is not None:
        codes = codes.copy()
        codes[missing] = MISSING_CODE
    pad = np.zeros((m, nb * 4), dtype=np.uint8)
    pad[:, :n] = codes
    pad = pad.reshape(m, nb, 4)
    packed = pad[:, :, 0] | (pad[:, :, 1] << 2) | (pad[:, :, 2] << 4) | (pad[:, :, 3] << 6)
    return bytes([0x6C, 0x1B, 0x01]) + packed.astype(np.uint8).tobytes()


def write_plink(prefix, geno, missing=None, n_chrom=10, seed=1):
    """Write prefix.bed/.bim/.fam for an (n_snp, n_id) dosage matrix."""
    m, n = geno.shape
    with open(prefix + ".bed", "wb") as f:
        f.write(pack_bed(geno, missing))
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    per = (m + n_chrom - 1) // n_chrom
    with open(prefix + ".bim", "w") as f:
        for j in range(m):
            chrom = j // per + 1
            bp = (j % per) * 10000 + 1000 + int(rng.integers(0, 5000))
            f.write("%d\tsnp%d\t%.3f\t%d\tA\tG\n" % (chrom, j, bp / 1e6, bp))
    with open(prefix + ".fam", "w") as f:
        for i in range(n):
            f.write("F%d I%d 0 0 0 -9\n" % (i // 10, i))


def simulate_phenotype(geno, var=(0.4, 0.2, 0.4), seed=2, extra=None):
    """y = 1 + sqrt(sA) L_A z1 + sqrt(sAA) L_AA z2 + sqrt(se) e, with K_A built as in
    gmat/gmatrix/gmatrix.py:53-66 (no diagonal boost) and K_AA = K_A o K_A.

    ``extra`` optionally gives additional (K, variance) pairs (e.g. D, AxD, DxD)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    g = geno.T.astype(np.float64)
    n = g.shape[0]
    p = g.sum(axis=0) / (2 * n)
    x = g - 2 * p
    ka = x @ x.T / np.sum(2 * p * (1 - p))
    comps = [(ka, var[0]), (ka * ka, var[1])]
    if extra:
        comps += list(extra)
    y = np.ones(n)
    for k, s in comps:
        L = np.linalg.cholesky(k + 1e-4 * np.eye(n))
        y += np.sqrt(s) * (L @ rng.standard_normal(n))
    y += np.sqrt(var[-1]) * rng.standard_normal(n)
    return y


def write_pheno(path, fam_prefix_ids, y, covar=None):
    """Pheno file in the layout of design_matrix.py:7-13: FID IID 1 [covariates] y."""
    with open(path, "w") as f:
        for i, (fid, iid) in enumerate(fam_prefix_ids):
            cols = [fid, iid, "1"]
            if covar is not None:
                cols += ["%.6g" % v for v in covar[i]]
            cols.append("%.10g" % y[i])
            f.write(" ".join(cols) + "\n")


def make_cohort(prefix, n_id, n_snp, seed=1, with_pheno=True, var=(0.4, 0.2, 0.4)):
    """Generate and write a full cohort: prefix.{bed,bim,fam} and prefix.pheno."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    geno = simulate_genotypes(n_id, n_snp, seed=seed)
    write_plink(prefix, geno, seed=seed)
    if with_pheno:
        y = simulate_phenotype(geno, var=var, seed=seed + 1)
        ids = [("F%d" % (i // 10), "I%d" % i) for i in range(n_id)]
        write_pheno(prefix + ".pheno", ids, y)
    return geno
