"""Full-triangle audit of the certified screens: over EVERY pair of a cohort, the screened scan
(prefilter -> low-rank spectral screen -> pair screen -> exact fp64 refine) returns exactly the
hits of the exhaustive scan (level GMAT_SCREEN_NONE: every pair refined, the reference's
computation remma_epiAA.py:71-82 / remma_epiAD.py:68-80 / remma_epiDD.py:68-79), with
byte-identical eff / var / chi / p.  The exhaustive scan itself is checked against the oracle on
a few rows, on up to 20,000 of its hits all over the triangle and on a random sample of its non-hits.  tools/full_triangle.py runs the same audit on the full configs[2] cohort.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_ID = 2000


def _cohort(m, seed):
    from gmat_amd import _native as N, synth
    from gmat_amd.plink import Geno
    from gmat_amd.uvlmm.uvlmm_varcom import projection
    from scipy.sparse import identity
    lib = N.ensure_device()
    geno = synth.simulate_genotypes(N_ID, m, seed=seed)
    body = np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8)
    g = Geno(body=body, n_id=N_ID, n_snp=m)
    ka = np.empty((N_ID, N_ID))
    sc = ctypes.c_double()
    N.check(lib.gmat_grm(g.handle, 0, 0.001, N.ptr(ka), ctypes.byref(sc)), "gmat_grm")
    kd = np.empty((N_ID, N_ID))
    N.check(lib.gmat_grm(g.handle, 1, 0.001, N.ptr(kd), ctypes.byref(sc)), "gmat_grm")
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    y = np.ones(N_ID)
    for k, s in ((ka, 0.4), (ka * ka, 0.2)):
        y += np.sqrt(s) * (np.linalg.cholesky(k + 1e-4 * np.eye(N_ID)) @ rng.standard_normal(N_ID))
    y += np.sqrt(0.4) * rng.standard_normal(N_ID)
    gl = [ka, kd, ka * ka, ka * kd, kd * kd]
    pvp, py = projection(y, np.ones((N_ID, 1)), identity(N_ID, format="csr"), gl, [0.3, 0.1, 0.1, 0.05, 0.05, 0.4])
    return geno, g, pvp, py


def _same(a, b):
    assert a[0].size == b[0].size, (a[0].size, b[0].size)
    for x, y in zip(a, b):
        assert x.dtype == y.dtype
        np.testing.assert_array_equal(x.view(np.uint64) if x.dtype == np.float64 else x,
                                      y.view(np.uint64) if y.dtype == np.float64 else y)


@pytest.fixture(scope="module")
def aa_cohort():
    geno, g, pvp, py = _cohort(6000, 41)
    yield geno, g, pvp, py
    g.close()


@pytest.fixture(scope="module")
def small_cohort():
    geno, g, pvp, py = _cohort(3000, 43)
    yield geno, g, pvp, py
    g.close()


def _audit(g, pvp, py, kind, p_cuts):
    from gmat_amd import _native as N
    from gmat_amd.remma._scan import EpiPlan
    m = g.m
    rows = np.arange(m if kind == "AD" else m - 1, dtype=np.int64)
    with EpiPlan(g, pvp, py) as plan:
        assert plan.lowrank_rank() > 0
        exh = plan.scan(kind, rows, max(p_cuts), n_slice=N.GMAT_SCREEN_NONE)
        st = plan.stats()
        assert st["pairs"] == (m * m if kind == "AD" else m * (m - 1) // 2)
        assert st["n_slice"] == N.GMAT_SCREEN_NONE
        for p_cut in p_cuts:
            sel = exh[5] < p_cut
            exp = tuple(a[sel] for a in exh)
            for ns in (0, -1):  # automatic level (low-rank screen at small p_cut), fp6 quadratic form
                got = plan.scan(kind, rows, p_cut, n_slice=ns)
                _same(got, exp)
    return exh


def _certificates(g, pvp, py, kind, pairs):
    """exact var >= each screen's certified lower bound (gmat_epi_audit) on every listed pair"""
    from gmat_amd.remma._scan import EpiPlan
    with EpiPlan(g, pvp, py) as plan:
        _, var, _, _ = plan.pairs(kind, pairs)
        lb = plan.audit(kind, pairs)
    worst = {}
    for col, name in ((0, "prefilter"), (1, "lowrank")):
        pos = lb[:, col] > 0
        assert pos.sum() > 0.1 * pairs.shape[0], (name, pos.sum())
        r = var[pos] / lb[pos, col]
        assert r.min() >= 1.0, (name, float(r.min()))
        worst[name] = float(r.min())
    print("min exact var / certified bound:", worst)


def test_full_triangle_aa(aa_cohort):
    geno, g, pvp, py = aa_cohort
    exh = _audit(g, pvp, py, "AA", (1e-5, 1e-3))
    rng = np.random.default_rng(5)
    i = rng.integers(0, g.m - 1, 8000)
    j = rng.integers(0, g.m, 8000)
    near = np.column_stack([exh[0], exh[1]])[exh[5] >= 1e-5]
    _certificates(g, pvp, py, "AA", np.vstack([np.column_stack([i, j])[i < j], near]))
    assert np.sum(exh[5] < 1e-5) >= 1 and exh[0].size > 1000, exh[0].size
    # the exhaustive level itself against the oracle (rows at both ends of the triangle)
    from oracle import gmat_oracle as O
    snp = np.ascontiguousarray(geno.T, dtype=np.float64)
    rows = np.array([0, 2999, 5997], dtype=np.int64)
    exp = O.epi_scan("AA", snp, pvp, py.reshape(-1, 1), snp_lst_0=rows, p_cut=1e-3)
    sel = np.isin(exh[0], rows)
    np.testing.assert_array_equal(np.column_stack([exh[0][sel], exh[1][sel]]), exp[:, :2].astype(np.int64))
    np.testing.assert_allclose(np.column_stack([exh[2][sel], exh[4][sel], exh[5][sel]]), exp[:, 2:], rtol=1e-8)
    # the exhaustive level's hits all over the triangle (up to 20,000 of them) against the oracle's pair
    # formula (remma_epiAA_pair.py:79-84), and a random sample of the other pairs: none of them a hit
    hits = np.column_stack([exh[0], exh[1]])
    pick = np.sort(np.random.default_rng(7).permutation(hits.shape[0])[:20000])
    eff_o, var_o, chi_o, p_o = O.epi_pair("AA", snp, pvp, py.reshape(-1, 1), hits[pick])
    assert np.all(p_o < 1e-3)
    np.testing.assert_allclose(np.column_stack([exh[2][pick], exh[3][pick], exh[4][pick], exh[5][pick]]),
                               np.column_stack([eff_o, var_o, chi_o, p_o]), rtol=1e-8)
    sample = np.column_stack([i, j])[i < j]
    sample = sample[~np.isin(sample[:, 0] * g.m + sample[:, 1], hits[:, 0] * g.m + hits[:, 1])]
    p_s = O.epi_pair("AA", snp, pvp, py.reshape(-1, 1), sample)[3]
    # (a monomorphic SNP gives var 0 and a NaN p, as in the reference: not a hit either)
    assert sample.shape[0] > 3000 and not np.any(p_s < 1e-3), (sample.shape[0], float(np.nanmin(p_s)))


@pytest.mark.parametrize("kind", ["AD", "DD"])
def test_full_triangle_ad_dd(small_cohort, kind):
    geno, g, pvp, py = small_cohort
    exh = _audit(g, pvp, py, kind, (1e-5, 1e-3))
    assert exh[0].size > 100, exh[0].size
    rng = np.random.default_rng(6)
    i = rng.integers(0, g.m, 4000)
    j = rng.integers(0, g.m, 4000)
    sel = (i < j) if kind == "DD" else np.ones(i.size, bool)
    _certificates(g, pvp, py, kind, np.vstack([np.column_stack([i, j])[sel], np.column_stack([exh[0], exh[1]])]))
    if kind == "AD":  # i == j pairs are part of the exhaustive AD scan
        from gmat_amd import _native as N
        from gmat_amd.remma._scan import EpiPlan
        with EpiPlan(g, pvp, py) as plan:
            d = plan.scan("AD", np.arange(5, dtype=np.int64), 1.0, n_slice=N.GMAT_SCREEN_NONE)
        assert d[0].size > 0 and np.any(d[0] == d[1])


def test_recorded_exhaustive_hit_set_still_applies():
    """bench.py checks every step against the recorded exhaustive hit set of its cohort
    (tests/golden/cfg3_exhaustive_hits_AA_2000x50000.npz) only while the cohort fingerprint (per-SNP
    counts, P, Py) matches: a change that moves a bit of P (the projection's Cholesky and inverse)
    silently turns that check off, so it fails here instead."""
    import os
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    import bench
    from tools.full_triangle import cohort_fingerprint
    rec = np.load(os.path.join(repo, bench.EXHAUSTIVE_HITS))
    _, g, pvp, py, _, _ = bench.build_inputs(2000, 50000, 1, np.array([0.4, 0.2, 0.4]), 0, 1)
    try:
        assert bytes(rec["fingerprint"]).hex() == cohort_fingerprint(g, pvp, py)
    finally:
        g.close()
