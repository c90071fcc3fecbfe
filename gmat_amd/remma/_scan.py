"""Shared host logic of the epistasis scans (AA / AD / DD, exact, parallel parts, pairs).

The reference's per-row numpy loop (remma_epiAA.py:71-82 and siblings) is replaced by one
device scan plan (gmat_epi: genotype panel, P and Py resident in HBM) that returns the
hits; this module keeps the reference's argument handling, defaults, error conditions,
output files and row order.
"""
import ctypes
import functools
import os
import logging
import time

import numpy as np
from scipy.stats import chi2

from .. import _native as N
from .. import dist
from ..plink import count_lines
from ..uvlmm.uvlmm_varcom import projection

KINDS = {"AA": N.GMAT_AA, "AD": N.GMAT_AD, "DD": N.GMAT_DD}
SCAN_HEADER = "snp_0 snp_1 eff chi p_val"
PAIR_HEADER = "snp_0 snp_1 eff var chi p"
N_SLICE = 3  # slices kept; each scan uses 1, 2 or 3 by p_cut (gmat_epi_scan n_slice=0)



@functools.lru_cache(maxsize=64)
def _chi_cut(p_cut):
    """chi2(1) quantile of p_cut (scipy's isf costs ~50 us: cached, the multi-GPU steps are ~3 ms)"""
    return float(chi2.isf(p_cut, 1)) if p_cut < 1 else 0.0

class EpiPlan:
    """gmat_epi handle: a genotype panel plus Z'PZ and Z'Py resident on the device."""

    def __init__(self, geno, pvp, py, n_slice=N_SLICE, state=None):
        """state: the spectral state of a plan for the same P (export_state() of another rank's
        plan); the eigendecomposition and certificate searches are then skipped."""
        self._lib = N.ensure_device()
        self.geno = geno
        pvp = N.f64(pvp)
        py = N.f64(np.asarray(py).reshape(-1))
        if pvp.shape != (geno.n, geno.n) or py.size != geno.n:
            raise ValueError("P is %s and Py has %d entries for %d genotyped individuals"
                             % (pvp.shape, py.size, geno.n))
        h = ctypes.c_void_p()
        if state is None:
            N.check(self._lib.gmat_epi_create(ctypes.byref(h), geno.handle, N.ptr(pvp), N.ptr(py), int(n_slice)),
                    "gmat_epi_create")
        else:
            st = np.ascontiguousarray(state, dtype=np.uint8)
            N.check(self._lib.gmat_epi_create_with(ctypes.byref(h), geno.handle, N.ptr(pvp), N.ptr(py), int(n_slice),
                                                   N.ptr(st), st.size), "gmat_epi_create_with")
        self._h = h

    def export_state(self):
        """The plan's spectral state as bytes (uint8 array) for EpiPlan(..., state=...)."""
        need = ctypes.c_int64()
        N.check(self._lib.gmat_epi_export(self._h, None, 0, ctypes.byref(need)), "gmat_epi_export")
        buf = np.zeros(need.value, dtype=np.uint8)
        N.check(self._lib.gmat_epi_export(self._h, N.ptr(buf), buf.size, ctypes.byref(need)), "gmat_epi_export")
        return buf

    def scan(self, kind, rows, p_cut, n_slice=0):
        """Hits (i, j, eff, var, chi, p) with p < p_cut over first-SNP rows `rows`
        (strictly increasing), sorted by (i, j).  n_slice picks the certified screen in front of
        the exact refine (gmat_epi_scan); N.GMAT_SCREEN_NONE refines every pair (the reference's
        computation, remma_epiAA.py:71-82) -- the audit of the screens."""
        rows = N.i64(rows)
        n_hits = ctypes.c_int64()
        chi_cut = _chi_cut(float(p_cut))
        N.check(self._lib.gmat_epi_scan(self._h, KINDS[kind], N.ptr(rows), rows.size, float(p_cut), chi_cut,
                                        int(n_slice), ctypes.byref(n_hits)), "gmat_epi_scan")
        k = n_hits.value
        out = [np.zeros(k, np.int64), np.zeros(k, np.int64)] + [np.zeros(k) for _ in range(4)]
        N.check(self._lib.gmat_epi_hits(self._h, k, *[N.ptr(a) for a in out]), "gmat_epi_hits")
        return tuple(out)

    def pairs(self, kind, pairs):
        pairs = N.i64(np.asarray(pairs).reshape(-1, 2))
        k = pairs.shape[0]
        out = [np.zeros(k) for _ in range(4)]
        N.check(self._lib.gmat_epi_pairs(self._h, KINDS[kind], N.ptr(pairs), k, *[N.ptr(a) for a in out]),
                "gmat_epi_pairs")
        return tuple(out)

    def audit(self, kind, pairs):
        """Certified lower bounds of e'Pe the screens test with, evaluated exactly for the listed
        pairs: columns (prefilter bound, low-rank bound, |e|^2, 1'e, |Q'e|^2); compare with
        pairs()' exact var (a ratio var / bound < 1 would be a certificate bug)."""
        pairs = N.i64(np.asarray(pairs).reshape(-1, 2))
        out = np.zeros((pairs.shape[0], 5))
        N.check(self._lib.gmat_epi_audit(self._h, KINDS[kind], N.ptr(pairs), pairs.shape[0], N.ptr(out)),
                "gmat_epi_audit")
        return out

    def stats(self):
        s = np.zeros(10)
        N.check(self._lib.gmat_epi_stats(self._h, N.ptr(s)), "gmat_epi_stats")
        keys = ("pairs", "candidates", "int8_ops", "screen_s", "refine_s", "side_s", "total_s", "launches",
                "n_slice", "bound_coef")
        return dict(zip(keys, s.tolist()))

    def kernel_stats(self):
        """Per-kernel accounting of the last low-rank-level scan (gmat_epi_kernel_stats)."""
        s = np.zeros(8)
        N.check(self._lib.gmat_epi_kernel_stats(self._h, N.ptr(s)), "gmat_epi_kernel_stats")
        keys = ("prefilter_s", "prefilter_launches", "prefilter_ops", "screen_s", "screen_launches", "screen_ops",
                "flush_s", "live_pairs")
        return dict(zip(keys, s.tolist()))

    def kernel_stats_ext(self):
        """The candidate kernels of the last scan (gmat_epi_kernel_stats_ext): seconds, launches and pairs
        of pair_side, pair_mx, refine and refine_side."""
        s = np.zeros(12)
        cnt = ctypes.c_int()
        N.check(self._lib.gmat_epi_kernel_stats_ext(self._h, N.ptr(s), s.size, ctypes.byref(cnt)),
                "gmat_epi_kernel_stats_ext")
        out = {}
        for k, name in enumerate(("pair_side", "pair_mx", "refine", "refine_side")):
            out[name] = {"s": float(s[3 * k]), "launches": float(s[3 * k + 1]), "pairs": float(s[3 * k + 2])}
        return out

    def setup_stats(self):
        """Plan setup seconds (gmat_epi_setup_stats): create total, prefilter certificate,
        eigendecomposition, low-rank certificate, slices/residual bounds, coding builds, and
        the number of Cholesky factorisations the certificates ran."""
        s = np.zeros(8)
        N.check(self._lib.gmat_epi_setup_stats(self._h, N.ptr(s)), "gmat_epi_setup_stats")
        keys = ("create_s", "prefilter_cert_s", "eigen_s", "lowrank_cert_s", "slices_bounds_s", "coding_s",
                "cholesky_count", "covariate_directions")
        return dict(zip(keys, s.tolist()))

    def lowrank_rank(self):
        """Rank of the plan's low-rank spectral screen (0: scans use the fp6 quadratic form)."""
        return int(self.info()["lowrank_rank"])

    def info(self):
        """Screen certificates and the prefilter's tile shape (gmat_epi_info)."""
        s = np.zeros(8)
        N.check(self._lib.gmat_epi_info(self._h, N.ptr(s)), "gmat_epi_info")
        keys = ("lowrank_rank", "lowrank_lam", "prefilter_mu", "n_pad", "pf_tile_rows", "pf_tile_cols",
                "pf_stage_dma_bytes", "pf_tile_record_bytes")
        return dict(zip(keys, s.tolist()))

    def layout(self):
        """How the plan holds its panel (gmat_epi_layout): SNP segments (1 = one plan), SNPs per segment,
        whether the plan is exhaustive-only (no screens past 8,192 individuals), and n_snp."""
        s = np.zeros(4, np.int64)
        N.check(self._lib.gmat_epi_layout(self._h, N.ptr(s)), "gmat_epi_layout")
        return {"segments": int(s[0]), "segment_snps": int(s[1]), "exhaustive_only": bool(s[2]), "n_snp": int(s[3])}

    def close(self):
        if getattr(self, "_h", None):
            self._lib.gmat_epi_destroy(self._h)
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


# wall seconds of the phases of the last run_scan call in this process (bench.py's end-to-end leg):
# projection (V, P, Py), decode (.bed read, checked, decoded on the device), plan (certificates),
# scan (the device scan, hits on the host), write (the hits file)
LAST_PHASES = {}


def open_plan(y, xmat, zmat, gmat_lst, var_com, bed_file, phases=None):
    """P / Py on the device (remma_epiAA.py:33-49), genotype panel decoded on the device.
    As a rank of a multi-rank job (dist.job): P / Py computed on rank 0 and broadcast, the panel read
    shard by shard and all-gathered, the plan's spectral state computed on rank 0 and imported by the
    other ranks (dist.shared_plan)."""
    phases = {} if phases is None else phases
    logging.info("Calculate the phenotypic covariance matrix and inversion")
    t0 = time.perf_counter()
    pvp, py = dist.root_call(projection, y, xmat, zmat, gmat_lst, var_com)
    t1 = time.perf_counter()
    geno = dist.load_geno(bed_file)
    t2 = time.perf_counter()
    phases["projection"], phases["decode"] = t1 - t0, t2 - t1
    if geno.n != pvp.shape[0]:
        geno.close()
        raise ValueError("Z has %d individuals, the .fam has %d" % (pvp.shape[0], geno.n))
    plan = dist.shared_plan(geno, pvp, py)
    phases["plan"] = time.perf_counter() - t2
    return plan


def format_rows(cols, n_float):
    """Rows as pandas DataFrame.to_csv writes them: ints, then float64 reprs (the Python statement
    of what append_rows writes natively)."""
    i, j = cols[0], cols[1]
    fl = cols[2:2 + n_float]
    return "".join("%d %d %s\n" % (a, b, " ".join(repr(float(v[t])) for v in fl)) for t, (a, b) in
                   enumerate(zip(i.tolist(), j.tolist())))


def append_rows(path, cols, n_float):
    """Append format_rows(cols, n_float) to the file at path through the library's C++ writer
    (gmat_append_hit_rows: same bytes, ~30x faster than the Python formatting)."""
    lib = N.load()
    i, j = N.i64(cols[0]), N.i64(cols[1])
    fl = [N.f64(v) for v in cols[2:2 + n_float]] + [None] * (4 - n_float)
    N.check(lib.gmat_append_hit_rows(os.fsencode(path), i.size, N.ptr(i), N.ptr(j), n_float, *[N.ptr(v) for v in fl]),
            "gmat_append_hit_rows")


def resolve_rows(kind, num_snp, snp_lst_0):
    """Default and range check of snp_lst_0 (remma_epiAA.py:63-68; AD: remma_epiAD.py:66-72)."""
    hi = num_snp if kind == "AD" else num_snp - 1
    if snp_lst_0 is None:
        return np.arange(hi, dtype=np.int64)
    rows = np.asarray(list(snp_lst_0), dtype=np.int64)
    if rows.size and (rows.max() > hi - 1 or rows.min() < 0):
        logging.error("snp_lst_0 is out of range!")
        raise ValueError("snp_lst_0 is out of range!")
    return rows


def _no_hits():
    return (np.zeros(0, np.int64), np.zeros(0, np.int64)) + tuple(np.zeros(0) for _ in range(4))


def run_scan(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, snp_lst_0, p_cut, out_file):
    """_remma_epiXX: header, then the hits of each row of snp_lst_0 in list order (the
    reference appends each row's hits with j ascending).
    As a multi-rank job (dist.job): the rows are sharded over the ranks (the folded split of the
    whole triangle, dist.rank_rows, or equal pair counts of a given list), the hits are merged on
    rank 0 and rank 0 alone writes out_file -- the bytes a single process writes."""
    rank, ws = dist.job()
    if rank == 0:
        with open(out_file, "w") as f:
            f.write(SCAN_HEADER + "\n")
    num_snp = count_lines(bed_file + ".bim")
    rows = resolve_rows(kind, num_snp, snp_lst_0)
    phases = {}
    plan = open_plan(y, xmat, zmat, gmat_lst, var_com, bed_file, phases)
    try:
        uniq = np.unique(rows)
        mine = dist.shard_rows(kind, num_snp, uniq, rank, ws)
        t0 = time.perf_counter()
        local = plan.scan(kind, mine, p_cut) if mine.size else _no_hits()
        phases["scan"] = time.perf_counter() - t0
        logging.info("Running time: Clock time, {:.5f} sec.".format(phases["scan"]))
        logging.info("scan stats: %s" % plan.stats())
    finally:
        t0 = time.perf_counter()
        plan.close()
        plan.geno.close()
        phases["release"] = time.perf_counter() - t0
    if ws > 1:
        t0 = time.perf_counter()
        local = dist.gather_hits(local)
        phases["gather"] = time.perf_counter() - t0
    if rank == 0:
        hi, hj, eff, var, chi, p = local
        if rows.size == uniq.size and np.all(np.diff(rows) > 0):
            order = np.arange(hi.size)
        else:  # replay the caller's row order (and duplicates) like the reference's loop
            starts = np.searchsorted(hi, uniq, side="left")
            ends = np.searchsorted(hi, uniq, side="right")
            pos = np.searchsorted(uniq, rows)
            order = np.concatenate([np.arange(starts[k], ends[k]) for k in pos]) if rows.size else np.zeros(0, int)
        t0 = time.perf_counter()
        append_rows(out_file, [hi[order], hj[order], eff[order], chi[order], p[order]], 3)
        phases["write"] = time.perf_counter() - t0
    if ws > 1:
        dist.barrier()  # out_file is complete when any rank returns
    LAST_PHASES.clear()
    LAST_PHASES.update(phases)
    return 0


def parallel_rows(num_snp, parallel, kind):
    """The triangle-folded part `parallel=[N, k]` (remma_epiAA.py:125-139; AD extends part 1
    to num_snp, remma_epiAD.py:134-140)."""
    n_part, k = int(parallel[0]), int(parallel[1])
    s = int(num_snp / (2 * n_part))
    p0, p1 = (k - 1) * s, k * s
    p2, p3 = (2 * n_part - k) * s, (2 * n_part - k + 1) * s
    if k == 1:
        p3 = num_snp if kind == "AD" else num_snp - 1
    return list(range(p0, p1)) + list(range(p2, p3))


def run_parallel(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, parallel, p_cut, out_file):
    logging.info("Parallel: " + str(parallel[0]) + ", " + str(parallel[1]))
    num_snp = count_lines(bed_file + ".bim")
    rows = parallel_rows(num_snp, parallel, kind)
    return run_scan(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, rows, p_cut,
                    out_file + "." + str(parallel[1]))


def read_pair_file(snp_pair_file):
    """First two columns of every line after the first (pd.read_csv(skiprows=1), :72-75)."""
    out = []
    with open(snp_pair_file) as f:
        f.readline()
        for line in f:
            a = line.split()
            if len(a) >= 2:
                out.append((int(a[0]), int(a[1])))
    return np.array(out, dtype=np.int64).reshape(-1, 2)


_PAIR_REC = np.dtype([("eff", "<f8"), ("var", "<f8"), ("chi", "<f8"), ("p", "<f8")])


def run_pairs(kind, y, xmat, zmat, gmat_lst, var_com, bed_file, snp_pair_file, max_test_pair, p_cut, out_file):
    """_remma_epiXX_pair (remma_epiAA_pair.py:16-92): exact statistics of the listed pairs,
    rows with p < p_cut in file order, columns snp_0 snp_1 eff var chi p.  The reference tests
    max_test_pair pairs at a time and stops at the first chunk holding an out-of-range SNP (the
    earlier chunks' rows are written, then ValueError).
    As a multi-rank job: the valid prefix of the list is cut into contiguous equal runs, one per rank
    (each tested max_test_pair at a time), the statistics are gathered in list order on rank 0, and
    rank 0 alone writes out_file."""
    rank, ws = dist.job()
    pairs = read_pair_file(snp_pair_file)
    num_snp = count_lines(bed_file + ".bim")
    step = max(1, int(max_test_pair))
    n_ok = pairs.shape[0]
    for t0 in range(0, pairs.shape[0], step):
        chunk = pairs[t0:t0 + step]
        if chunk.size and (chunk.max() > num_snp - 1 or chunk.min() < 0):
            n_ok = t0
            break
    plan = open_plan(y, xmat, zmat, gmat_lst, var_com, bed_file)
    if rank == 0:
        with open(out_file, "w") as f:
            f.write(PAIR_HEADER + "\n")
    try:
        b = dist.split_weighted(np.ones(n_ok), ws)
        mine = pairs[b[rank]:b[rank + 1]]
        rec = np.zeros(mine.shape[0], dtype=_PAIR_REC)
        for t0 in range(0, mine.shape[0], step):
            res = plan.pairs(kind, mine[t0:t0 + step])
            for name, col in zip(_PAIR_REC.names, res):
                rec[name][t0:t0 + step] = col
            if ws == 1:  # a single process writes chunk by chunk, as the reference
                keep = rec["p"][t0:t0 + step] < p_cut
                sub = mine[t0:t0 + step]
                append_rows(out_file, [sub[keep, 0], sub[keep, 1]] +
                            [rec[nm][t0:t0 + step][keep] for nm in _PAIR_REC.names], 4)
    finally:
        plan.close()
        plan.geno.close()
    if ws > 1:
        rec = dist.gather_records(rec)
        if rank == 0:
            keep = rec["p"] < p_cut
            sub = pairs[:n_ok]
            append_rows(out_file, [sub[keep, 0], sub[keep, 1]] + [rec[nm][keep] for nm in _PAIR_REC.names], 4)
        dist.barrier()
    if n_ok < pairs.shape[0]:
        logging.error("snp_pair is out of range!")
        raise ValueError("snp_pair is out of range!")
    return 0
