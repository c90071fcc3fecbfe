"""Parity of the HIP product path (gmat_amd via libgmat_hip.so) with the reference.

Checked against the golden fixtures the reference produced (tests/golden/) and against the
CPU oracle on the same seeded inputs.  Bars: SNP-pair indices and hit sets exact;
variance components, effects, variances, chi and p within 1e-5 relative (north star), in
practice ~1e-10 because the reported statistics are recomputed in fp64.
"""
import gzip
import hashlib
import io
import json
import os
import shutil

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TINY = os.path.join(GOLD, "tiny")
MOUSE = os.path.join(GOLD, "mouse")
RTOL = 1e-5


def _copy(src_prefix, names, dst_dir, new_prefix):
    for ext in names:
        shutil.copy(src_prefix + ext, os.path.join(dst_dir, new_prefix + ext))
    return os.path.join(dst_dir, new_prefix)


@pytest.fixture(scope="module")
def tiny_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("tiny")
    bed = _copy(os.path.join(TINY, "tiny"), (".bed", ".bim", ".fam", ".pheno"), str(d), "tiny")
    return bed


@pytest.fixture(scope="module")
def mouse_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("mouse")
    for f in ("plink.bed", "plink.bim", "plink.fam", "pheno"):
        shutil.copy(os.path.join(MOUSE, f), str(d))
    return os.path.join(str(d), "plink")


def _hits(path):
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rt") as f:
        lines = f.read().splitlines()
    body = [l for l in lines[1:] if l.strip()]
    arr = np.loadtxt(io.StringIO("\n".join(body)), ndmin=2) if body else np.zeros((0, 5))
    return lines[0], arr


def _cmp_hits(got_file, exp_file, ncol_float=3):
    hg, g = _hits(got_file)
    he, e = _hits(exp_file)
    assert hg == he
    assert g.shape == e.shape, (g.shape, e.shape)
    np.testing.assert_array_equal(g[:, :2], e[:, :2])
    np.testing.assert_allclose(g[:, 2:], e[:, 2:], rtol=RTOL, atol=1e-300)
    return g, e


# ---------------------------------------------------------------- GRM


def test_agmat_tiny(tiny_dir):
    from gmat_amd.gmatrix import agmat, dgmat_as
    ref = np.load(os.path.join(TINY, "tiny_ref.npz"))
    meta = json.load(open(os.path.join(TINY, "text_outputs.json")))
    k, kinv = agmat(tiny_dir, inv=True)
    np.testing.assert_allclose(k, ref["agmat"], rtol=1e-11, atol=1e-12)
    np.testing.assert_allclose(kinv, ref["agmat_inv"], rtol=1e-7, atol=1e-8)
    d, _ = dgmat_as(tiny_dir)
    np.testing.assert_allclose(d, ref["dgmat"], rtol=1e-11, atol=1e-12)
    # text formats: same layout; values may differ in the last digits of %.18e
    for ext in (".agrm0", ".dgrm_as0"):
        exp_head = meta[ext]["head"][0].split()
        got_head = open(tiny_dir + ext).readline().split()
        assert len(exp_head) == len(got_head) == 150
        np.testing.assert_allclose([float(v) for v in got_head], [float(v) for v in exp_head], rtol=1e-11,
                                   atol=1e-12)
    agmat(tiny_dir, out_fmt="row_col_val")
    agmat(tiny_dir, out_fmt="id_id_val")
    for ext in (".agrm1", ".agrm2"):
        got = open(tiny_dir + ext).read().splitlines()
        assert len(got) == 150 * 151 // 2
        for gl, el in zip(got[:3], meta[ext]["head"]):
            ga, ea = gl.split(), el.split()
            assert ga[:2] == ea[:2]
            assert abs(float(ga[2]) - float(ea[2])) <= 1e-11 * max(1.0, abs(float(ea[2])))


def test_agmat_mouse_summary(mouse_dir):
    from gmat_amd.gmatrix import agmat, dgmat_as
    for name, fn in (("agmat", agmat), ("dgmat_as", dgmat_as)):
        ref = np.load(os.path.join(MOUSE, name + ".npz"))
        k, _ = fn(mouse_dir)
        np.testing.assert_allclose(np.diag(k), ref["diag"], rtol=1e-11)
        np.testing.assert_allclose(k[0], ref["row0"], rtol=1e-9, atol=1e-11)
        np.testing.assert_allclose(k[ref["ia"], ref["ib"]], ref["val"], rtol=1e-9, atol=1e-11)
        assert abs(np.trace(k) - float(ref["trace"])) < 1e-8
        np.testing.assert_array_equal(k, k.T)


def test_spd_inverse_random():
    from gmat_amd.gmatrix import spd_inverse
    rng = np.random.default_rng(0)
    for n in (1, 7, 64, 65, 200, 777):
        a = rng.standard_normal((n, n + 5))
        a = a @ a.T + n * np.eye(n)
        np.testing.assert_allclose(spd_inverse(a), np.linalg.inv(a), rtol=1e-9, atol=1e-12)


# ---------------------------------------------------------------- REML


def test_reml_tiny(tiny_dir):
    from gmat_amd.uvlmm import wemai_multi_gmat, _wemai_multi_gmat
    ref = np.load(os.path.join(TINY, "tiny_ref.npz"))
    a = ref["agmat"]
    var = wemai_multi_gmat(tiny_dir + ".pheno", tiny_dir, [a, a * a], out_file=tiny_dir + ".var")
    np.testing.assert_allclose(var, ref["var"], rtol=1e-7)
    np.testing.assert_allclose(_wemai_multi_gmat.last_history, ref["hist"], rtol=1e-6)


def test_reml_mouse_known_answer(mouse_dir):
    from gmat_amd.uvlmm import wemai_multi_gmat
    ref = np.load(os.path.join(MOUSE, "reml.npz"))
    a = np.load(os.path.join(MOUSE, "agmat.npz"))
    from gmat_amd.gmatrix import agmat, dgmat_as
    ka, _ = agmat(mouse_dir)
    kd, _ = dgmat_as(mouse_dir)
    var2 = wemai_multi_gmat(mouse_dir.replace("plink", "pheno"), mouse_dir, [ka, ka * ka], out_file=mouse_dir + ".v2")
    np.testing.assert_allclose(var2, ref["var2"], rtol=1e-6)
    np.testing.assert_allclose(var2, [0.06289206, 0.07641075, 0.08121168], rtol=1e-6)  # remma_cpu.py:178
    var5 = wemai_multi_gmat(mouse_dir.replace("plink", "pheno"), mouse_dir, [ka, kd, ka * ka, ka * kd, kd * kd],
                            out_file=mouse_dir + ".v5")
    np.testing.assert_allclose(var5, ref["var5"], rtol=1e-6)
    del a


# ---------------------------------------------------------------- scans


@pytest.mark.parametrize("kind", ["AA", "AD", "DD"])
def test_tiny_every_pair(tiny_dir, kind, tmp_path):
    """p_cut=1: every testable pair (NaN pairs of monomorphic / all-het SNPs dropped)."""
    import gmat_amd.remma as R
    ref = np.load(os.path.join(TINY, "tiny_ref.npz"))
    a = ref["agmat"]
    fn = getattr(R, "remma_epi" + kind)
    out = str(tmp_path / ("epi" + kind))
    fn(tiny_dir + ".pheno", tiny_dir, [a, a * a], ref["var"], p_cut=1.0, out_file=out)
    _cmp_hits(out, os.path.join(TINY, "epi%s_all.gz" % kind))


def _mouse_grms(mouse_dir):
    from gmat_amd.gmatrix import agmat, dgmat_as
    ka, _ = agmat(mouse_dir)
    kd, _ = dgmat_as(mouse_dir)
    return ka, kd


def test_mouse_scans(mouse_dir, tmp_path):
    import gmat_amd.remma as R
    ref = np.load(os.path.join(MOUSE, "reml.npz"))
    ka, kd = _mouse_grms(mouse_dir)
    pheno = mouse_dir.replace("plink", "pheno")
    g2 = [ka, ka * ka]
    g5 = [ka, kd, ka * ka, ka * kd, kd * kd]
    for p_cut, name in ((1e-5, "epiAA_1e-5"), (1e-3, "epiAA_1e-3")):
        R.remma_epiAA(pheno, mouse_dir, g2, ref["var2"], p_cut=p_cut, out_file=str(tmp_path / name))
        _cmp_hits(str(tmp_path / name), os.path.join(MOUSE, name))
    R.remma_epiAD(pheno, mouse_dir, g5, ref["var5"], p_cut=1e-5, out_file=str(tmp_path / "ad"))
    _cmp_hits(str(tmp_path / "ad"), os.path.join(MOUSE, "epiAD_1e-5"))
    R.remma_epiDD(pheno, mouse_dir, g5, ref["var5"], p_cut=1e-5, out_file=str(tmp_path / "dd"))
    _cmp_hits(str(tmp_path / "dd"), os.path.join(MOUSE, "epiDD_1e-5"))


def test_mouse_covariates_keep_fast_path(mouse_dir):
    """The mouse pheno (intercept + 3 covariates): the plan certifies the prefilter with the
    covariate directions and builds the low-rank screen, so the golden scans above ran on the
    low-rank level (round 1 fell back to the fp6 quadratic form for every covariate design)."""
    from gmat_amd.remma._scan import open_plan
    from gmat_amd.uvlmm.design_matrix import design_matrix_wemai_multi_gmat
    ref = np.load(os.path.join(MOUSE, "reml.npz"))
    ka, _ = _mouse_grms(mouse_dir)
    y, x, z = design_matrix_wemai_multi_gmat(mouse_dir.replace("plink", "pheno"), mouse_dir)
    assert x.shape[1] == 4
    plan = open_plan(y, x, z, [ka, ka * ka], ref["var2"], mouse_dir)
    try:
        assert plan.setup_stats()["covariate_directions"] == 3
        assert plan.lowrank_rank() > 0
        plan.scan("AA", np.arange(plan.geno.m - 1), 1e-5)
        assert plan.stats()["n_slice"] == -1
    finally:
        plan.close()
        plan.geno.close()


def test_mouse_pairs_and_parallel(mouse_dir, tmp_path):
    import gmat_amd.remma as R
    ref = np.load(os.path.join(MOUSE, "reml.npz"))
    ka, _ = _mouse_grms(mouse_dir)
    pheno = mouse_dir.replace("plink", "pheno")
    g2 = [ka, ka * ka]
    R.remma_epiAA_pair(pheno, mouse_dir, g2, ref["var2"], os.path.join(MOUSE, "pairs5000"), p_cut=1.0,
                       out_file=str(tmp_path / "pair"))
    _cmp_hits(str(tmp_path / "pair"), os.path.join(MOUSE, "epiAA_pair5000"))
    for k in (1, 2, 3):
        R.remma_epiAA_parallel(pheno, mouse_dir, g2, ref["var2"], [3, k], p_cut=1e-4,
                               out_file=str(tmp_path / "par"))
        _cmp_hits(str(tmp_path / ("par.%d" % k)), os.path.join(MOUSE, "epiAA_par3_1e-4.%d" % k))
    shutil.copy(os.path.join(MOUSE, "epiAA_1e-3"), str(tmp_path / "hits"))
    R.annotation_snp_pos(str(tmp_path / "hits"), mouse_dir, p_cut=1e-4, dis=1000000)
    assert open(str(tmp_path / "hits.anno")).read() == open(os.path.join(MOUSE, "epiAA_1e-3.anno")).read()


# ---------------------------------------------------------------- larger sizes vs the oracle


@pytest.fixture(scope="module")
def synth_cohort(tmp_path_factory):
    from gmat_amd import synth
    d = tmp_path_factory.mktemp("synth")
    prefix = os.path.join(str(d), "c")
    geno = synth.make_cohort(prefix, 600, 3000, seed=7)
    return prefix, geno


def test_scan_vs_oracle_rows(synth_cohort):
    """A 600 x 3,000 cohort (n not a multiple of 128): GPU hits on stratified rows equal
    the oracle's row-by-row reference computation."""
    from oracle import gmat_oracle as O
    from gmat_amd.remma._scan import EpiPlan
    from gmat_amd.plink import Geno
    from gmat_amd.uvlmm.design_matrix import design_matrix_wemai_multi_gmat
    prefix, _ = synth_cohort
    snp = O.read_plink(prefix)
    ka = O.agmat(snp)
    y, x, col, nid = O.design_matrix(prefix + ".pheno", prefix)
    var = np.array([0.4, 0.2, 0.4])
    pvp, py = O.projection(y, x, col, nid, [ka, ka * ka], var)
    rows = np.array([0, 1, 2, 500, 1499, 2001, 2990, 2998])
    with Geno(prefix) as g, EpiPlan(g, pvp, py[:, 0]) as plan:
        for kind, p_cut, ns in (("AA", 5e-2, 0), ("DD", 5e-2, 0), ("AD", 5e-2, 0), ("AA", 0.5, 1), ("DD", 0.3, 1),
                                ("AD", 0.5, 1), ("AA", 1e-3, 1), ("AA", 0.5, -1), ("DD", 0.3, -1), ("AD", 0.5, -1),
                                ("AA", 1e-4, -1), ("AA", 1e-4, -2), ("AA", 0.5, -2), ("DD", 0.3, -2), ("AD", 0.5, -2),
                                ("DD", 1e-3, -2), ("AD", 1e-3, -2)):
            # forced single-slice screens at large p_cut put most pairs inside the bound's band
            hi, hj, eff, var_, chi, p = plan.scan(kind, rows, p_cut, n_slice=ns)
            exp = O.epi_scan(kind, snp, pvp, py, snp_lst_0=rows, p_cut=p_cut)
            assert hi.size == exp.shape[0], (kind, p_cut, ns, hi.size, exp.shape)
            np.testing.assert_array_equal(np.column_stack([hi, hj]), exp[:, :2].astype(np.int64))
            np.testing.assert_allclose(np.column_stack([eff, chi, p]), exp[:, 2:], rtol=1e-8, atol=1e-300)
            # the pair kernel gives the same numbers for the same pairs
            e2, v2, c2, p2 = plan.pairs(kind, np.column_stack([hi, hj]))
            np.testing.assert_array_equal(e2, eff)
            np.testing.assert_array_equal(p2, p)
    del design_matrix_wemai_multi_gmat


def test_scan_deterministic_and_row_split(synth_cohort):
    """Full triangle at p_cut=1e-3: identical results when run twice and when the rows are
    split into the reference's parallel parts (the multi-GPU sharding unit)."""
    from oracle import gmat_oracle as O
    from gmat_amd.remma._scan import EpiPlan, parallel_rows
    from gmat_amd.plink import Geno
    prefix, _ = synth_cohort
    snp = O.read_plink(prefix)
    ka = O.agmat(snp)
    y, x, col, nid = O.design_matrix(prefix + ".pheno", prefix)
    pvp, py = O.projection(y, x, col, nid, [ka, ka * ka], [0.4, 0.2, 0.4])
    m = snp.shape[1]
    with Geno(prefix) as g, EpiPlan(g, pvp, py[:, 0]) as plan:
        full = plan.scan("AA", np.arange(m - 1), 1e-3)
        st = plan.stats()
        assert st["pairs"] == m * (m - 1) // 2 and st["candidates"] >= full[0].size
        again = plan.scan("AA", np.arange(m - 1), 1e-3)
        for a, b in zip(full, again):
            np.testing.assert_array_equal(a, b)
        # the hit set does not depend on the screen level (-2: low-rank spectral screen, reported
        # as -1; -1: fp6 x fp4 MX quadratic form, reported as 0; 1-3: int8 slices)
        for ns, level in ((-2, -1), (-1, 0), (1, 1), (2, 2), (3, 3)):
            forced = plan.scan("AA", np.arange(m - 1), 1e-3, n_slice=ns)
            assert plan.stats()["n_slice"] == level, (ns, plan.stats())
            for a, b in zip(full, forced):
                np.testing.assert_array_equal(a, b)
        parts = [plan.scan("AA", np.array(sorted(parallel_rows(m, [4, k], "AA"))), 1e-3) for k in (1, 2, 3, 4)]
        cat = [np.concatenate([p[t] for p in parts]) for t in range(6)]
        order = np.lexsort((cat[1], cat[0]))
        for a, b in zip(full, cat):
            np.testing.assert_array_equal(a, b[order])


def test_repeated_records_and_prediction(tiny_dir, tmp_path):
    """Z != I: REML and the exact AA scan on repeated, unordered
    records; wemai_multi_gmat_pred with record-less genotyped ids (.var and .rand_eff)."""
    import gmat_amd.remma as R
    from gmat_amd.uvlmm import wemai_multi_gmat, wemai_multi_gmat_pred
    ref = np.load(os.path.join(TINY, "tiny_ref.npz"))
    rep = np.load(os.path.join(TINY, "rep_ref.npz"))
    a = ref["agmat"]
    pheno = os.path.join(TINY, "rep.pheno")
    var = wemai_multi_gmat(pheno, tiny_dir, [a, a * a], out_file=str(tmp_path / "v"))
    np.testing.assert_allclose(var, rep["var"], rtol=1e-6)
    R.remma_epiAA(pheno, tiny_dir, [a, a * a], rep["var"], p_cut=0.05, out_file=str(tmp_path / "aa"))
    _cmp_hits(str(tmp_path / "aa"), os.path.join(TINY, "rep_epiAA"))
    out = str(tmp_path / "pred")
    pv = wemai_multi_gmat_pred(os.path.join(TINY, "rep_pred.pheno"), tiny_dir, [a, a * a], out_file=out)
    np.testing.assert_allclose(pv, rep["pred_var"], rtol=1e-6)
    np.testing.assert_allclose(np.loadtxt(out + ".var"), rep["pred_var"], rtol=1e-6)
    re = np.loadtxt(out + ".rand_eff")
    assert re.shape == (150, 2)
    np.testing.assert_allclose(re, rep["rand_eff"], rtol=1e-5, atol=1e-10)


def test_scan_large_n(tmp_path):
    """n = 4,133 (n_pad 4,224 > 4,096: deeper K-loops, larger epilogue sums) on a 400-SNP
    cohort: every kind on stratified rows vs the oracle; also the plan's pair kernel."""
    from oracle import gmat_oracle as O
    from gmat_amd import synth
    from gmat_amd.remma._scan import EpiPlan
    from gmat_amd.plink import Geno
    prefix = str(tmp_path / "big")
    synth.make_cohort(prefix, 4133, 400, seed=17)
    snp = O.read_plink(prefix)
    ka = O.agmat(snp)
    y, x, col, nid = O.design_matrix(prefix + ".pheno", prefix)
    pvp, py = O.projection(y, x, col, nid, [ka, ka * ka], [0.4, 0.2, 0.4])
    rows = np.array([0, 3, 150, 398])
    with Geno(prefix) as g, EpiPlan(g, pvp, py[:, 0]) as plan:
        for kind, ns in (("AA", 0), ("DD", 0), ("AD", 0), ("AA", -1), ("AD", -1), ("AA", -2), ("DD", -2), ("AD", -2)):
            hi, hj, eff, var_, chi, p = plan.scan(kind, rows, 0.2, n_slice=ns)
            exp = O.epi_scan(kind, snp, pvp, py, snp_lst_0=rows, p_cut=0.2)
            assert hi.size == exp.shape[0] and hi.size > 20, (kind, hi.size, exp.shape)
            np.testing.assert_array_equal(np.column_stack([hi, hj]), exp[:, :2].astype(np.int64))
            np.testing.assert_allclose(np.column_stack([eff, chi, p]), exp[:, 2:], rtol=1e-8, atol=1e-300)
