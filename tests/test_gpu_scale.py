"""Parity at the BASELINE configurations' own sizes (BASELINE.json configs[1], configs[2]) and
the hardware check of the low-rank screen's fp32 accumulation bound.

* cfg3 (2,000 x 50,000, p_cut 1e-5, the headline cohort of bench.py): the exhaustive scan's hit
  set on stratified first-SNP rows equals the oracle's exact fp64 computation
  (remma_epiAA.py:71-82) at every screen level -- low-rank spectral screen, fp6 x fp4 quadratic
  form, int8 slices -- for AA, and on the automatic level for DD and AD (i == j included).
* cfg2 (2,000 x 20,000): agmat's full matrix and the 2-GRM REML ([A, AxA], uvlmm_varcom.py:41-99)
  against the oracle.
* The screen's bound |c~_r - c_r| <= eta_r = 2^-24 |Q_r|_1 (8 n_pad + 400) (epi_plan.hip lr_setup) on
  adversarial operands (same sign, w = 4, n_pad up to 8,192, block scales 2^16 apart).
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N3, M3, SEED3 = 2000, 50000, 1  # bench.py's cohort


def _fp6_value(code):
    s = (code >> 5) & 1
    e = (code >> 3) & 3
    m = code & 7
    v = np.where(e > 0, np.ldexp(1.0 + m / 8.0, e - 1), m / 8.0)
    return np.where(s == 1, -v, v)


@pytest.mark.parametrize("n_steps", [2, 32, 128])
def test_mx_accumulation_bound(n_steps):
    """v_mfma_scale_f32_32x32x64_f8f6f4 chains (the low-rank screen's accumulation) on
    adversarial same-sign operands: the observed fp32 error stays within eta_r."""
    from gmat_amd import _native as N
    lib = N.ensure_device()
    rng = np.random.default_rng(n_steps)
    worst = 0.0
    for pattern in range(3):
        codes = np.zeros((n_steps, 32, 2, 32), dtype=np.uint8)
        scales = np.zeros((n_steps, 32, 2), dtype=np.uint8)
        if pattern == 0:  # largest magnitudes, random mantissas, one scale
            codes[:] = 24 + rng.integers(0, 8, codes.shape)
            scales[:] = 127
        elif pattern == 1:  # big blocks then tiny increments: every add rounds
            codes[:] = 8 + rng.integers(0, 24, codes.shape)
            big = (np.arange(n_steps) % 4 == 0)[:, None, None]
            scales[:] = np.where(big, 127 + 12, 127 - 4)
        else:  # geometric growth of the partial sums
            codes[:] = 9 + rng.integers(0, 23, codes.shape)
            scales[:] = (120 + (np.arange(n_steps) * 16) // n_steps)[:, None, None]
        out = np.zeros((32, 32), dtype=np.float32)
        N.check(lib.gmat_probe_mx_accum(n_steps, N.ptr(codes), N.ptr(scales), N.ptr(out)), "gmat_probe_mx_accum")
        vals = _fp6_value(codes.astype(np.int64)) * np.ldexp(1.0, scales.astype(np.int64) - 127)[..., None]
        exact = 4.0 * vals.sum(axis=(0, 2, 3))  # per row; exact in fp64 (few significant bits each)
        n_pad = 64 * n_steps
        l1 = np.abs(vals).sum(axis=(0, 2, 3))
        eta = 2.0 ** -24 * l1 * (8.0 * n_pad + 400.0) * 1.01
        err = np.abs(out.astype(np.float64) - exact[:, None])
        assert np.all(err <= eta[:, None]), (pattern, float((err / eta[:, None]).max()))
        for c in range(1, 32):  # every column is the same product
            np.testing.assert_array_equal(out[:, c], out[:, 0])
        worst = max(worst, float((err / eta[:, None]).max()))
    print("worst observed error / eta = %.3g" % worst)


# ------------------------------------------------------------------------------------ cfg3


@pytest.fixture(scope="module")
def cfg3():
    from gmat_amd import _native as N, synth
    from gmat_amd.plink import Geno
    from gmat_amd.uvlmm.uvlmm_varcom import projection
    from scipy.sparse import identity
    lib = N.ensure_device()
    geno = synth.simulate_genotypes(N3, M3, seed=SEED3)
    body = np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8)
    g = Geno(body=body, n_id=N3, n_snp=M3)
    ka = np.empty((N3, N3))
    sc = ctypes.c_double()
    N.check(lib.gmat_grm(g.handle, 0, 0.001, N.ptr(ka), ctypes.byref(sc)), "gmat_grm")
    rng = np.random.Generator(np.random.PCG64(SEED3 + 1))
    y = np.ones(N3)
    for k, s in ((ka, 0.4), (ka * ka, 0.2)):
        y += np.sqrt(s) * (np.linalg.cholesky(k + 1e-4 * np.eye(N3)) @ rng.standard_normal(N3))
    y += np.sqrt(0.4) * rng.standard_normal(N3)
    pvp, py = projection(y, np.ones((N3, 1)), identity(N3, format="csr"), [ka, ka * ka], [0.4, 0.2, 0.4])
    snp = np.ascontiguousarray(geno.T, dtype=np.float64)
    yield g, snp, pvp, py
    g.close()


def test_cfg3_stratified_rows_vs_oracle(cfg3):
    """Headline cohort: identical hit sets on 24 stratified rows for every screen level."""
    from oracle import gmat_oracle as O
    from gmat_amd.remma._scan import EpiPlan
    g, snp, pvp, py = cfg3
    rows = np.unique(np.concatenate([np.linspace(0, M3 - 2, 22).astype(np.int64), [1, 24999]]))
    exp_all = O.epi_scan("AA", snp, pvp, py.reshape(-1, 1), snp_lst_0=rows, p_cut=1e-3)
    with EpiPlan(g, pvp, py) as plan:
        assert plan.lowrank_rank() > 0
        for p_cut in (1e-5, 1e-3):
            exp = exp_all[exp_all[:, 4] < p_cut]
            # 0: the automatic level (the low-rank screen at p_cut <= 1e-4, int8 slices above);
            # -2: low-rank (reported -1); -1: fp6 x fp4 quadratic form (reported 0); 1: int8
            for ns, level in ((0, None), (-2, -1), (-1, 0), (1, 1)):
                hi, hj, eff, var, chi, p = plan.scan("AA", rows, p_cut, n_slice=ns)
                lv = plan.stats()["n_slice"]
                assert level is None or ((lv == level) if level <= 0 else (lv >= level)), (ns, lv)
                assert hi.size == exp.shape[0], (p_cut, ns, hi.size, exp.shape)
                np.testing.assert_array_equal(np.column_stack([hi, hj]), exp[:, :2].astype(np.int64))
                np.testing.assert_allclose(np.column_stack([eff, chi, p]), exp[:, 2:], rtol=1e-8, atol=1e-300)
        assert exp_all[exp_all[:, 4] < 1e-5].shape[0] >= 1 and exp_all.shape[0] > 200


@pytest.mark.parametrize("kind", ["DD", "AD"])
def test_cfg3_dd_ad_rows_vs_oracle(cfg3, kind):
    from oracle import gmat_oracle as O
    from gmat_amd.remma._scan import EpiPlan
    g, snp, pvp, py = cfg3
    rows = np.array([0, 17, 20001, 49998], dtype=np.int64)
    exp = O.epi_scan(kind, snp, pvp, py.reshape(-1, 1), snp_lst_0=rows, p_cut=1e-3)
    with EpiPlan(g, pvp, py) as plan:
        hi, hj, eff, var, chi, p = plan.scan(kind, rows, 1e-3)
    assert hi.size == exp.shape[0] and hi.size > 10, (hi.size, exp.shape)
    np.testing.assert_array_equal(np.column_stack([hi, hj]), exp[:, :2].astype(np.int64))
    np.testing.assert_allclose(np.column_stack([eff, chi, p]), exp[:, 2:], rtol=1e-8, atol=1e-300)


# ------------------------------------------------------------------------------------ cfg2


def test_cfg2_grm_and_reml_vs_oracle(tmp_path):
    """configs[1]: 2,000 x 20,000 agmat (full matrix) and the 2-GRM REML vs the oracle."""
    from oracle import gmat_oracle as O
    from gmat_amd import synth
    from gmat_amd.gmatrix import agmat
    from gmat_amd.uvlmm import wemai_multi_gmat, _wemai_multi_gmat
    prefix = str(tmp_path / "cfg2")
    synth.make_cohort(prefix, 2000, 20000, seed=12)
    k, _ = agmat(prefix, out_fmt="npy")
    snp = O.read_plink(prefix)
    np.testing.assert_allclose(k, O.agmat(snp), rtol=1e-10, atol=1e-12)
    var = wemai_multi_gmat(prefix + ".pheno", prefix, [k, k * k], out_file=prefix + ".var")
    hist = _wemai_multi_gmat.last_history
    y, x, col, nid = O.design_matrix(prefix + ".pheno", prefix)
    oh = []
    ovar = O.wemai_multi_gmat(y, x, col, nid, [k, k * k], history=oh)
    assert len(oh) == hist.shape[0], (len(oh), hist.shape)
    np.testing.assert_allclose(var, ovar, rtol=1e-6)
    np.testing.assert_allclose(hist, np.array(oh), rtol=1e-6)
    assert os.path.exists(prefix + ".var")


def test_cfg3_covariates_vs_oracle(cfg3):
    """The headline cohort with intercept + 3 covariates (binary, integer-valued, binary -- the
    mouse example's layout): the plan keeps the certified fast path (prefilter with the three
    covariate directions, low-rank screen) and the hit sets equal the oracle's."""
    from oracle import gmat_oracle as O
    from gmat_amd.remma._scan import EpiPlan
    from gmat_amd.uvlmm.uvlmm_varcom import projection
    from scipy.sparse import identity
    g, snp, _, _ = cfg3
    rng = np.random.default_rng(31)
    x = np.column_stack([np.ones(N3), rng.integers(0, 2, N3), rng.integers(90, 130, N3), rng.integers(0, 2, N3)])
    ka = O.agmat(snp[:, :4000])
    y = 1.0 + x[:, 1] * 0.3 + x[:, 2] * 0.01 + rng.standard_normal(N3)
    pvp, py = projection(y, x.astype(float), identity(N3, format="csr"), [ka, ka * ka], [0.4, 0.2, 0.4])
    rows = np.unique(np.linspace(0, M3 - 2, 12).astype(np.int64))
    exp_all = O.epi_scan("AA", snp, pvp, py.reshape(-1, 1), snp_lst_0=rows, p_cut=1e-3)
    with EpiPlan(g, pvp, py) as plan:
        st = plan.setup_stats()
        assert st["covariate_directions"] == 3, st
        assert plan.lowrank_rank() > 0
        for p_cut in (1e-5, 1e-3):
            exp = exp_all[exp_all[:, 4] < p_cut]
            for ns, level in ((-2, -1), (-1, 0)):
                hi, hj, eff, var, chi, p = plan.scan("AA", rows, p_cut, n_slice=ns)
                assert plan.stats()["n_slice"] == level
                assert hi.size == exp.shape[0], (p_cut, ns, hi.size, exp.shape)
                np.testing.assert_array_equal(np.column_stack([hi, hj]), exp[:, :2].astype(np.int64))
                np.testing.assert_allclose(np.column_stack([eff, chi, p]), exp[:, 2:], rtol=1e-8, atol=1e-300)
        for kind in ("DD", "AD"):
            exp = O.epi_scan(kind, snp, pvp, py.reshape(-1, 1), snp_lst_0=rows[:4], p_cut=1e-3)
            hi, hj, eff, var, chi, p = plan.scan(kind, rows[:4], 1e-3, n_slice=-2)
            assert hi.size == exp.shape[0], (kind, hi.size, exp.shape)
            np.testing.assert_array_equal(np.column_stack([hi, hj]), exp[:, :2].astype(np.int64))


def test_grm_and_inverse_at_cfg5_n():
    """n = 5,000 (configs[4]'s individuals; ceil(n/4) = 1,250 bytes per SNP row: unaligned dword
    reads of the packed rows): agmat / dgmat_as against the oracle on 3,000 SNPs, and the SPD
    inverse of V-like matrices at n = 2,049 and 5,000 against numpy."""
    import ctypes
    from oracle import gmat_oracle as O
    from gmat_amd import _native as N, synth
    from gmat_amd.gmatrix import spd_inverse
    from gmat_amd.plink import Geno
    lib = N.ensure_device()
    n, m = 5000, 3000
    geno = synth.simulate_genotypes(n, m, seed=21)
    body = np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8)
    snp = np.ascontiguousarray(geno.T, dtype=np.float64)
    with Geno(body=body, n_id=n, n_snp=m) as g:
        for kind, ref in ((0, O.agmat), (1, O.dgmat_as)):
            k = np.empty((n, n))
            sc = ctypes.c_double()
            N.check(lib.gmat_grm(g.handle, kind, 0.001, N.ptr(k), ctypes.byref(sc)), "gmat_grm")
            np.testing.assert_allclose(k, ref(snp), rtol=1e-10, atol=1e-12)
    rng = np.random.default_rng(2)
    for nn in (2049, 5000):
        a = rng.standard_normal((nn, 300))
        v = a @ a.T / 300 + 0.5 * np.eye(nn)
        vi = spd_inverse(v)
        np.testing.assert_allclose(vi, np.linalg.inv(v), rtol=1e-8, atol=1e-10)
