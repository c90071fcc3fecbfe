"""BASELINE configs[4] at its own size: 5,000 individuals x 100,000 SNPs, the 5-GRM model
[A, D, AxA, AxD, DxD] (uvlmm_varcom.py:8-104, remma_epiAD.py:16-91, remma_epiDD.py:16-90).

* epiDD (j > i) and epiAD (every j, i == j included, both orientations) on stratified rows: the
  exhaustive GPU scan's hits are checked against the oracle's exact fp64 statistics on a sample
  of 3,000 second SNPs per row that contains every GPU hit (so every reported hit is an oracle hit
  with the oracle's numbers, and no sampled pair the oracle calls a hit is missing);
* the same with a candidate buffer far smaller than one launch's candidates (escalation and
  buffer growth, GMAT_CAND_CAP);
* the first two REML iterations of the 5-GRM model at n = 5,000 against the oracle's.
n_pad = 5,120, 2 m n_pad = 1.02e9 (the 32-bit buffer offsets' range, epi.hip gmat_epi_create).
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N5, M5, SEED5 = 5000, 100000, 5


@pytest.fixture(scope="module")
def cfg5():
    from gmat_amd import _native as N, synth
    from gmat_amd.plink import Geno
    from gmat_amd.uvlmm.uvlmm_varcom import projection
    from scipy.sparse import identity
    lib = N.ensure_device()
    geno, _ = synth.simulate_genotype_shard(N5, M5, 0, M5, seed=SEED5)
    g = Geno(body=np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8), n_id=N5, n_snp=M5)
    mats = []
    for kind in (0, 1):
        k = np.empty((N5, N5))
        sc = ctypes.c_double()
        N.check(lib.gmat_grm(g.handle, kind, 0.001, N.ptr(k), ctypes.byref(sc)), "gmat_grm")
        mats.append(k)
    a, d = mats
    gl = [a, d, a * a, a * d, d * d]
    rng = np.random.default_rng(SEED5)
    y = 1.0 + (np.linalg.cholesky(a + 1e-3 * np.eye(N5)) @ rng.standard_normal(N5)) * 0.5 + rng.standard_normal(N5)
    var = np.array([0.3, 0.1, 0.1, 0.05, 0.05, 0.4])
    pvp, py = projection(y, np.ones((N5, 1)), identity(N5, format="csr"), gl, var)
    yield g, geno, gl, y, pvp, py
    g.close()


def _oracle_sample(kind, geno, pvp, py, i, js):
    """Exact (eff, var, chi, p) of pairs (i, js) from the columns involved only (the codings'
    centring is per SNP, so a column subset gives the same numbers)."""
    from oracle import gmat_oracle as O
    cols = np.unique(np.concatenate([[i], js]))
    snp = np.ascontiguousarray(geno[cols].T, dtype=np.float64)
    loc = {c: t for t, c in enumerate(cols.tolist())}
    pairs = np.array([[loc[i], loc[j]] for j in js.tolist()], dtype=np.int64)
    return O.epi_pair(kind, snp, pvp, py.reshape(-1, 1), pairs)


def _check_rows(plan, kind, geno, pvp, py, rows, p_cut, rng):
    hi, hj, eff, var, chi, p = plan.scan(kind, rows, p_cut)
    n_checked = 0
    for i in rows.tolist():
        sel = hi == i
        lo_j = 0 if kind == "AD" else i + 1
        cand = np.arange(lo_j, M5)
        js = np.unique(np.concatenate([hj[sel], rng.choice(cand, min(3000, cand.size), replace=False),
                                       [i] if kind == "AD" else []]).astype(np.int64))
        oe, ov, oc, op = _oracle_sample(kind, geno, pvp, py, i, js)
        exp_hit = js[op < p_cut]
        np.testing.assert_array_equal(hj[sel], exp_hit)
        k = np.searchsorted(js, hj[sel])
        np.testing.assert_allclose(eff[sel], oe[k], rtol=1e-8)
        np.testing.assert_allclose(p[sel], op[k], rtol=1e-8)
        n_checked += js.size
    return hi.size, n_checked


@pytest.mark.parametrize("kind", ["DD", "AD"])
def test_cfg5_scan_sampled_vs_oracle(cfg5, kind):
    from gmat_amd.remma._scan import EpiPlan
    g, geno, gl, y, pvp, py = cfg5
    rng = np.random.default_rng(1 if kind == "DD" else 2)
    rows = np.array([0, 33333, 77777, M5 - 2], dtype=np.int64)
    with EpiPlan(g, pvp, py) as plan:
        assert plan.lowrank_rank() > 0
        n_hits, n_checked = _check_rows(plan, kind, geno, pvp, py, rows, 1e-3, rng)
    assert n_hits > 10 and n_checked > 8000


def test_cfg5_candidate_overflow_growth(cfg5):
    """A 2,048-pair candidate buffer against ~400k AD pairs at p_cut 0.02: every launch
    overflows, escalates to the int8 slices and finally grows the buffer; the hits equal those
    of a plan with the default buffer, and the sampled oracle check holds."""
    from gmat_amd.remma._scan import EpiPlan
    g, geno, gl, y, pvp, py = cfg5
    rows = np.array([5, 50005, 99990], dtype=np.int64)
    with EpiPlan(g, pvp, py) as plan:
        ref = plan.scan("AD", rows, 0.02)
    os.environ["GMAT_CAND_CAP"] = "2048"
    try:
        with EpiPlan(g, pvp, py) as plan:
            got = plan.scan("AD", rows, 0.02)
            assert plan.stats()["n_slice"] >= 1
            for a, b in zip(ref, got):
                np.testing.assert_array_equal(a, b)
            assert got[0].size > 2048
            _check_rows(plan, "AD", geno, pvp, py, rows[:1], 0.02, np.random.default_rng(3))
    finally:
        del os.environ["GMAT_CAND_CAP"]


def test_cfg5_reml_first_iterations_vs_oracle(cfg5):
    from oracle import gmat_oracle as O
    from gmat_amd.uvlmm.uvlmm_varcom import _wemai_multi_gmat
    from scipy.sparse import identity
    g, geno, gl, y, pvp, py = cfg5
    var = _wemai_multi_gmat(y, np.ones((N5, 1)), identity(N5, format="csr"), gl, maxiter=2)
    hist = _wemai_multi_gmat.last_history
    oh = []
    O.wemai_multi_gmat(y.reshape(-1, 1), np.ones((N5, 1)), np.arange(N5), N5, gl, maxiter=2, history=oh)
    np.testing.assert_allclose(hist, np.array(oh), rtol=1e-7)
    assert var.size == 6


def test_cfg5_reml_to_the_end_vs_oracle(cfg5):
    """The 5-GRM REML at n = 5,000 run to convergence or the reference's maxiter (200): the oracle,
    started from the GPU's iterate k - 2 (uvlmm_varcom.py:107 `init`), reproduces the last two
    iterates -- the whole trajectory is the reference's, not only its first steps."""
    from oracle import gmat_oracle as O
    from gmat_amd.uvlmm.uvlmm_varcom import _wemai_multi_gmat
    from scipy.sparse import identity
    g, geno, gl, y, pvp, py = cfg5
    var = _wemai_multi_gmat(y, np.ones((N5, 1)), identity(N5, format="csr"), gl, maxiter=200)
    hist = _wemai_multi_gmat.last_history
    k = hist.shape[0]
    assert k >= 3
    print("REML iterations %d (converged: %s), var %s" % (k, k < 200, np.array2string(var, precision=5)))
    oh = []
    O.wemai_multi_gmat(y.reshape(-1, 1), np.ones((N5, 1)), np.arange(N5), N5, gl, init=hist[k - 3], maxiter=2,
                       history=oh)
    np.testing.assert_allclose(np.array(oh), hist[k - 2:], rtol=1e-6)
    np.testing.assert_allclose(var, hist[-1], rtol=0, atol=0)
