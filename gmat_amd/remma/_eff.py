"""Host logic of the approximate pipeline: the effect-only screen (_eff, _maf_eff) and the
approximate tests built on it (_approx, _maf_approx), for AA / AD / DD.

The screen itself is the device kernel behind the reference's C symbols
(``remma_epi{AA,AD,DD}(_maf)_eff_cpu``, include/gmat_remma_eff.h), called through ctypes exactly
where the reference calls its cffi module (remma_epiAA_eff.py:64-80); everything around it --
defaults, range checks, the threshold eff_cut = sqrt(chi2.isf(p_cut, 1) * var_app), the
``.temp`` file and its chi_app / p_app post-processing, the random-pair variance estimate and
the final merge -- follows the reference's Python (remma_epiAA_eff.py:20-96,
remma_epiAA_maf_eff.py:20-104, remma_epiAA_approx.py:10-101, remma_epiAA_maf_approx.py:11-90
and the AD / DD copies).
"""
import logging
import os
import time

import numpy as np
import pandas as pd
from scipy.stats import chi2

from .. import _native as N
from .. import dist
from ..plink import Geno, count_lines
from ..uvlmm.design_matrix import design_matrix_wemai_multi_gmat
from ..uvlmm.uvlmm_varcom import projection
from ._scan import parallel_rows, run_pairs
from .random_pair import random_pair, random_pairAD

_SYM = {"AA": "remma_epiAA_eff_cpu", "AD": "remma_epiAD_eff_cpu", "DD": "remma_epiDD_eff_cpu"}
_SYM_MAF = {"AA": "remma_epiAA_maf_eff_cpu", "AD": "remma_epiAD_maf_eff_cpu", "DD": "remma_epiDD_maf_eff_cpu"}


def _py(y, xmat, zmat, gmat_lst, var_com):
    """Z'Py (remma_epiAA_eff.py:36-51); P stays on the device side of gmat_projection.  Computed on
    rank 0 of a multi-rank job and broadcast."""
    logging.info("Calculate the phenotypic covariance matrix and inversion")
    return N.f64(dist.root_call(lambda: projection(y, xmat, zmat, gmat_lst, var_com)[1]))


def _rows(kind, num_snp, snp_lst_0):
    """Default list and range check (AA/DD remma_epiAA_eff.py:57-62; AD remma_epiAD_eff.py:56-61)."""
    hi = num_snp if kind == "AD" else num_snp - 1
    if snp_lst_0 is None:
        return np.arange(hi, dtype=np.longlong)
    rows = np.array(list(snp_lst_0), dtype=np.longlong)
    if rows.size and (rows.max() > hi - 1 or rows.min() < 0):
        logging.error("snp_lst_0 is out of range!")
        raise ValueError("snp_lst_0 is out of range!")
    return rows


def _enc(s):
    return s.encode("ascii")


def eff_stats():
    """(pairs, hits, device seconds, text seconds) of the last screen in this process."""
    s = np.zeros(4)
    N.check(N.load().gmat_eff_stats(N.ptr(s)), "gmat_eff_stats")
    return dict(zip(("pairs", "hits", "device_s", "write_s"), s.tolist()))


def _screen(sym, args, temp_file):
    lib = N.ensure_device()
    t0 = time.perf_counter()
    rc = getattr(lib, sym)(*args)
    if rc != 1:
        N.check(rc if rc < 0 else N.GMAT_E_ARG, sym)
    logging.info("Running time: Clock time, {:.5f} sec. {}".format(time.perf_counter() - t0, eff_stats()))


def _screen_parts(kind, sym, make_args, num_snp, rows, temp_file):
    """The effect screen over `rows` into temp_file.  As a multi-rank job: the row list is cut into
    contiguous runs of about equal pair counts, rank r screens run r into temp_file.part<r>, and rank 0
    joins the parts in rank order (one header) -- the file a single process writes, byte for byte."""
    rank, ws = dist.job()
    if ws == 1:
        _screen(sym, make_args(rows, temp_file), temp_file)
        return
    b = dist.split_weighted(dist.row_pairs(kind, num_snp, rows), ws)
    mine = np.ascontiguousarray(rows[b[rank]:b[rank + 1]])
    part = "%s.part%d" % (temp_file, rank)
    _screen(sym, make_args(mine, part), part)
    dist.barrier()
    if rank == 0:
        with open(temp_file, "wb") as fout:
            for r in range(ws):
                name = "%s.part%d" % (temp_file, r)
                with open(name, "rb") as fin:
                    head = fin.readline()
                    if r == 0:
                        fout.write(head)
                    while True:
                        blk = fin.read(1 << 22)
                        if not blk:
                            break
                        fout.write(blk)
                os.remove(name)
    dist.barrier()


def _append_p(temp_file, out_file, deno):
    """The reference's post-processing loop (remma_epiAA_eff.py:85-96): each screened line gets
    chi_app = eff^2 / deno and p_app = chi2.sf(chi_app, 1), with eff re-read from the %g text.
    ``deno(i, j)`` gives the denominators of the rows (vectorised; same values, same text)."""
    logging.info("Add the approximate P values")
    with open(temp_file) as fin:
        head = fin.readline().strip()
        lines = [ln.split() for ln in fin]
    with open(out_file, "w") as fout:
        fout.write(head + " chi_app p_app\n")
        if lines:
            i = np.array([int(a[0]) for a in lines], dtype=np.int64)
            j = np.array([int(a[1]) for a in lines], dtype=np.int64)
            e = np.array([float(a[-1]) for a in lines])
            chi_app = e * e / deno(i, j)
            p_app = chi2.sf(chi_app, 1)
            fout.write("".join("%s %s %s\n" % (" ".join(a), repr(float(c)), repr(float(p)))
                               for a, c, p in zip(lines, chi_app.tolist(), p_app.tolist())))
    os.remove(temp_file)


def run_eff(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=None, var_app=1.0, p_cut=1.0e-5,
            out_file="epiAA_eff"):
    py = _py(y, xmat, zmat, gmat_lst, var_com)
    num_snp = count_lines(bed_file + ".bim")
    num_id = count_lines(bed_file + ".fam")
    rows = _rows(kind, num_snp, snp_lst_0)
    chi_cut = chi2.isf(p_cut, 1)
    eff_cut = np.sqrt(chi_cut * var_app)
    temp_file = out_file + ".temp"
    logging.info("Test")
    _screen_parts(kind, _SYM[kind], lambda r, tf: (_enc(bed_file), num_id, num_snp, N.ptr(r), r.size, N.ptr(py),
                                                   float(eff_cut), _enc(tf)), num_snp, rows, temp_file)
    dist.root_call(_append_p, temp_file, out_file, lambda i, j: var_app)
    return 0


def run_maf_eff(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=None, freq_i=None, freq_j=None,
                freq_deno=None, p_cut=1.0e-5, out_file="epiAA_maf_eff"):
    """_remma_epiXX_maf_eff: per-frequency-class thresholds eff_cut[fi*10 + fj] (111 entries).
    AA / DD pass the same ``freq`` as freq_i and freq_j, AD passes freqA, freqD."""
    py = _py(y, xmat, zmat, gmat_lst, var_com)
    num_snp = count_lines(bed_file + ".bim")
    num_id = count_lines(bed_file + ".fam")
    rows = _rows(kind, num_snp, snp_lst_0)
    if freq_i is None:
        freq_i = np.zeros((num_snp,), dtype=np.longlong)
    if freq_j is None:
        freq_j = np.zeros((num_snp,), dtype=np.longlong)
    if freq_deno is None:
        freq_deno = np.ones(111)
    freq_i = np.ascontiguousarray(freq_i, dtype=np.longlong)
    freq_j = np.ascontiguousarray(freq_j, dtype=np.longlong)
    chi_cut = chi2.isf(p_cut, 1)
    eff_cut = np.ascontiguousarray(np.sqrt(chi_cut * np.asarray(freq_deno, dtype=float)))
    if kind != "AD":
        # remma_epiAA_maf_eff.py:79 (written to the working directory)
        dist.root_call(np.savetxt, "eff_cut", eff_cut)
    temp_file = out_file + ".temp"
    logging.info("Test")

    def make_args(r, tf):
        if kind == "AD":
            return (_enc(bed_file), num_id, num_snp, N.ptr(r), r.size, N.ptr(py), N.ptr(freq_i), N.ptr(freq_j),
                    N.ptr(eff_cut), _enc(tf))
        return (_enc(bed_file), num_id, num_snp, N.ptr(r), r.size, N.ptr(py), N.ptr(freq_i), N.ptr(eff_cut), _enc(tf))

    _screen_parts(kind, _SYM_MAF[kind], make_args, num_snp, rows, temp_file)
    deno = np.asarray(freq_deno, dtype=float)
    dist.root_call(_append_p, temp_file, out_file, lambda i, j: deno[freq_i[i] * 10 + freq_j[j]])
    return 0


def _parallel_out(kind, bed_file, parallel, out_file):
    logging.info("Parallel: " + str(parallel[0]) + ", " + str(parallel[1]))
    num_snp = count_lines(bed_file + ".bim")
    return parallel_rows(num_snp, parallel, kind), out_file + "." + str(parallel[1])


def run_eff_parallel(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, var_app=1.0, p_cut=1.0e-5,
                     out_file="epiAA_eff_parallel"):
    rows, out = _parallel_out(kind, bed_file, parallel, out_file)
    return run_eff(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=rows, var_app=var_app,
                   p_cut=p_cut, out_file=out)


def run_maf_eff_parallel(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, freq_i=None, freq_j=None,
                         freq_deno=None, p_cut=1.0e-5, out_file="epiAA_maf_eff_parallel"):
    rows, out = _parallel_out(kind, bed_file, parallel, out_file)
    return run_maf_eff(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0=rows, freq_i=freq_i,
                       freq_j=freq_j, freq_deno=freq_deno, p_cut=p_cut, out_file=out)


# ---------------------------------------------------------------- approximate pipelines

def _pheno_pairs(kind, pheno_file, bed_file, gmat_lst, var_com, pair_file, out_file):
    """remma_epiXX_pair(..., p_cut=1) on a pair file (the random pairs, then the survivors)."""
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    return run_pairs(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, pair_file, 50000, 1, out_file)


@dist.on_root
def _random(kind, num_snp, out_file, num_pair, seed):
    fn = random_pairAD if kind == "AD" else random_pair
    return fn(num_snp, out_file=out_file, num_pair=num_pair, seed=seed)


@dist.on_root
def _merge(approx_file, exact_file, out_file):
    """remma_epiAA_approx.py:40-53: insert p_app before the exact p of every exact_p line."""
    logging.info("\n\n#####Merge the results#####")
    p_dct = {}
    with open(approx_file) as fin:
        for line in fin:
            arr = line.split()
            p_dct[" ".join(arr[:2])] = arr[-1]
    with open(exact_file) as fin, open(out_file, "w") as fout:
        for line in fin:
            arr = line.split()
            arr.insert(-1, p_dct[" ".join(arr[:2])])
            fout.write(" ".join(arr) + "\n")
    os.remove(approx_file)
    os.remove(exact_file)


@dist.on_root
def _median_var(random_file, pair_file):
    """Median exact variance of the random pairs (remma_epiAA_approx.py:24-27); both files removed."""
    res_df = pd.read_csv(random_file, header=0, sep=r"\s+")
    var_median = np.median(res_df["var"])
    os.remove(pair_file)
    os.remove(random_file)
    return var_median


def run_approx(kind, pheno_file, bed_file, gmat_lst, var_com, p_cut=1.0e-5, num_random_pair=100000,
               out_file="epiAA_approx", parallel=None, seed=None):
    """remma_epiXX_approx (remma_epiAA_approx.py:10-53) and its _parallel form (:56-101):
    median exact variance of random pairs -> effect screen with var_app = median -> exact
    re-test of the survivors -> merged file 'snp_0 snp_1 eff var chi p_app p'."""
    sfx = "" if parallel is None else "." + str(parallel[1])
    logging.info("\n\n#####Randomly select {:d} pairs, and test these SNP pairs#####".format(num_random_pair))
    num_snp = count_lines(bed_file + ".bim")
    rp = out_file + ".random_pair" + sfx
    _random(kind, num_snp, rp, num_random_pair, seed)
    _pheno_pairs(kind, pheno_file, bed_file, gmat_lst, var_com, rp, out_file + ".random" + sfx)
    var_median = _median_var(out_file + ".random" + sfx, rp)
    logging.info("\n\n#####Screen the epistatic effects and select top SNP pairs based on approximate test#####")
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    if parallel is None:
        run_eff(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, var_app=var_median, p_cut=p_cut,
                out_file=out_file + ".approx_p")
        final = out_file
    else:
        run_eff_parallel(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, var_app=var_median,
                         p_cut=p_cut, out_file=out_file + ".approx_p")
        final = out_file + sfx
    logging.info("\n\n#####Calculate exact p values for top SNP pairs#####")
    _pheno_pairs(kind, pheno_file, bed_file, gmat_lst, var_com, out_file + ".approx_p" + sfx,
                 out_file + ".exact_p" + sfx)
    _merge(out_file + ".approx_p" + sfx, out_file + ".exact_p" + sfx, final)
    return 0


@dist.on_root
def _freq_classes(kind, bed_file, out_file, sfx):
    """Frequency classes of remma_epiAA_maf_approx.py:32-41 (AA: minor allele frequency),
    remma_epiDD_maf_approx.py:33-44 (DD: heterozygosity) and remma_epiAD_maf_approx.py:33-50
    (AD: both), with their side files; sums are the device panel's exact integer counts."""
    geno = Geno(bed_file)
    try:
        n = geno.n
        dose = geno.sum_dose.astype(float)
        het = geno.n_het.astype(float)
    finally:
        geno.close()
    if kind == "AA":
        freq = 1 - dose / (2 * n)
        freq[freq > 0.5] = 1 - freq[freq > 0.5]
        np.savetxt(out_file + ".freq" + sfx, freq)
        freq = np.array(list(map(np.longlong, freq * 20)), dtype=np.longlong)
        return freq, freq
    freq_d = het / n
    freq_d[freq_d > 0.5] = 1 - freq_d[freq_d > 0.5]
    if kind == "DD":
        np.savetxt(out_file + ".heter" + sfx, freq_d)
        freq_d = np.array(freq_d * 20, dtype=np.longlong)
        return freq_d, freq_d
    freq_a = dose / (2 * n)
    freq_a[freq_a > 0.5] = 1 - freq_a[freq_a > 0.5]
    np.savetxt(out_file + ".maf" + sfx, freq_a)
    np.savetxt(out_file + ".heter" + sfx, freq_d)
    return np.array(freq_a * 20, dtype=np.longlong), np.array(freq_d * 20, dtype=np.longlong)


@dist.on_root
def _class_denominators(kind, random_file, freq_i, freq_j, deno_file):
    """Mean exact variance per (class_i, class_j) of the random pairs, both orientations for
    AA / DD (remma_epiAA_maf_approx.py:43-71), (A class of snp_0, D class of snp_1) for AD
    (remma_epiAD_maf_approx.py:51-75); unseen classes get the overall mean."""
    fi = [str(v) for v in freq_i.tolist()]
    fj = [str(v) for v in freq_j.tolist()]
    sums, counts = {}, {}
    with open(random_file) as fin:
        fin.readline()
        for line in fin:
            arr = line.split()
            a, b, v = int(arr[0]), int(arr[1]), float(arr[-3])
            keys = [fi[a] + " " + fj[b]] if kind == "AD" else [fi[a] + " " + fi[b], fi[b] + " " + fi[a]]
            for k in keys:
                counts[k] = counts.get(k, 0) + 1
                sums[k] = sums.get(k, 0.0) + v
    all_sum, all_count = 0, 0
    for k in counts:
        all_sum += sums[k]
        all_count += counts[k]
        sums[k] = sums[k] / counts[k]
    all_mean = all_sum / all_count
    freq_deno = np.ones(111)
    with open(deno_file, "w") as fout:
        for key1 in set(freq_i):
            for key2 in set(freq_j):
                k = " ".join([str(key1), str(key2)])
                if k not in sums:
                    sums[k] = all_mean
                fout.write(k + " " + str(sums[k]) + "\n")
                freq_deno[key1 * 10 + key2] = sums[k]
    return freq_deno


def run_maf_approx(kind, pheno_file, bed_file, gmat_lst, var_com, p_cut=1.0e-5, num_random_pair=100000,
                   out_file="epiAA_maf_approx", parallel=None, seed=None):
    """remma_epiXX_maf_approx and its _parallel form: class-wise variance denominators instead
    of one median, then the same screen / re-test / merge."""
    sfx = "" if parallel is None else "." + str(parallel[1])
    logging.info("\n\n#####Randomly select {:d} pairs, and test these SNP pairs#####".format(num_random_pair))
    num_snp = count_lines(bed_file + ".bim")
    rp = out_file + (".random_pairAD" if (kind == "AD" and parallel is None) else ".random_pair") + sfx
    _random(kind, num_snp, rp, num_random_pair, seed)
    _pheno_pairs(kind, pheno_file, bed_file, gmat_lst, var_com, rp, out_file + ".random" + sfx)
    dist.root_call(os.remove, rp)
    logging.info("\n\n#####Calcualte the approximate denominator for Wald chi-square test#####")
    freq_i, freq_j = _freq_classes(kind, bed_file, out_file, sfx)
    freq_deno = _class_denominators(kind, out_file + ".random" + sfx, freq_i, freq_j,
                                    out_file + ".freq_denominator" + sfx)
    logging.info("\n\n#####Screen the epistatic effects and select top SNP pairs based on approximate test#####")
    y, xmat, zmat = design_matrix_wemai_multi_gmat(pheno_file, bed_file)
    if parallel is None:
        run_maf_eff(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, freq_i=freq_i, freq_j=freq_j,
                    freq_deno=freq_deno, p_cut=p_cut, out_file=out_file + ".approx_p")
        final = out_file
    else:
        run_maf_eff_parallel(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, freq_i=freq_i,
                             freq_j=freq_j, freq_deno=freq_deno, p_cut=p_cut, out_file=out_file + ".approx_p")
        final = out_file + sfx
    logging.info("\n\n#####Calculate exact p values for top SNP pairs#####")
    _pheno_pairs(kind, pheno_file, bed_file, gmat_lst, var_com, out_file + ".approx_p" + sfx,
                 out_file + ".exact_p" + sfx)
    _merge(out_file + ".approx_p" + sfx, out_file + ".exact_p" + sfx, final)
    return 0
