"""Pin the CPU oracle (oracle/gmat_oracle.py) to the golden fixtures the reference produced.

These run without a GPU.  They make the oracle a trustworthy checker for the HIP path.
"""
import gzip
import hashlib
import io
import json
import os

import numpy as np
import pytest

from oracle import gmat_oracle as O

MOUSE_DATA = os.path.join(os.path.dirname(__file__), "golden", "mouse")
TINY = os.path.join(os.path.dirname(__file__), "golden", "tiny")


def _load_hits(path):
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rt") as f:
        lines = f.read().splitlines()
    if len(lines) <= 1:
        return lines[0], np.zeros((0, 5))
    return lines[0], np.loadtxt(io.StringIO("\n".join(lines[1:])), ndmin=2)


@pytest.fixture(scope="module")
def tiny():
    snp = O.read_plink(os.path.join(TINY, "tiny"))
    ref = np.load(os.path.join(TINY, "tiny_ref.npz"))
    y, x, col, nid = O.design_matrix(os.path.join(TINY, "tiny.pheno"), os.path.join(TINY, "tiny"))
    return snp, ref, (y, x, col, nid)


def test_tiny_grm(tiny):
    snp, ref, _ = tiny
    assert snp.shape == (150, 200)
    np.testing.assert_allclose(O.agmat(snp), ref["agmat"], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(O.dgmat_as(snp), ref["dgmat"], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(np.linalg.inv(O.agmat(snp)), ref["agmat_inv"], rtol=1e-8, atol=1e-9)


def test_tiny_reml(tiny):
    snp, ref, (y, x, col, nid) = tiny
    a = O.agmat(snp)
    hist = []
    var = O.wemai_multi_gmat(y, x, col, nid, [a, a * a], history=hist)
    np.testing.assert_allclose(var, ref["var"], rtol=1e-8)
    np.testing.assert_allclose(np.array(hist), ref["hist"], rtol=1e-6)


@pytest.mark.parametrize("kind", ["AA", "AD", "DD"])
def test_tiny_all_pairs(tiny, kind):
    snp, ref, (y, x, col, nid) = tiny
    a = O.agmat(snp)
    pvp, py = O.projection(y, x, col, nid, [a, a * a], ref["var"])
    got = O.epi_scan(kind, snp, pvp, py, p_cut=1.0)
    hdr, exp = _load_hits(os.path.join(TINY, "epi%s_all.gz" % kind))
    assert hdr == "snp_0 snp_1 eff chi p_val"
    # NaN statistics (monomorphic / all-het SNPs) are dropped exactly as the reference does
    assert got.shape == exp.shape
    np.testing.assert_array_equal(got[:, :2], exp[:, :2])
    np.testing.assert_allclose(got[:, 2:], exp[:, 2:], rtol=1e-9, atol=1e-12)


def test_mouse_grm_summary():
    snp = O.read_plink(os.path.join(MOUSE_DATA, "plink")) if os.path.exists(
        os.path.join(MOUSE_DATA, "plink.bed")) else None
    if snp is None:
        pytest.skip("mouse data is only present in the build container")
    for name, fn in (("agmat", O.agmat), ("dgmat_as", O.dgmat_as)):
        ref = np.load(os.path.join(MOUSE_DATA, name + ".npz"))
        k = fn(snp)
        np.testing.assert_allclose(np.diag(k), ref["diag"], rtol=1e-12)
        np.testing.assert_allclose(k[0], ref["row0"], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(k[ref["ia"], ref["ib"]], ref["val"], rtol=1e-10, atol=1e-12)
        assert abs(np.trace(k) - ref["trace"]) < 1e-9


def test_known_answer_reml_values():
    # the reference repo's only known answer: examples/remma/remma_cpu.py:178
    ref = np.load(os.path.join(MOUSE_DATA, "reml.npz"))
    np.testing.assert_allclose(ref["var2"], [0.06289206, 0.07641075, 0.08121168], rtol=1e-6)


def test_parallel_rows_cover():
    for kind, total in (("AA", 1406), ("AD", 1407)):
        for n_part in (1, 2, 3, 5, 8):
            rows = sum((O.parallel_rows(1407, [n_part, k], kind) for k in range(1, n_part + 1)), [])
            assert sorted(rows) == list(range(total))


def test_parallel_parts_match_golden():
    # the union of the three reference part files equals the subset of a full scan
    parts = []
    for k in (1, 2, 3):
        _, h = _load_hits(os.path.join(MOUSE_DATA, "epiAA_par3_1e-4.%d" % k))
        rows = set(O.parallel_rows(1407, [3, k]))
        assert all(int(i) in rows for i in h[:, 0])
        parts.append(h)
    allh = np.concatenate(parts)
    _, full = _load_hits(os.path.join(MOUSE_DATA, "epiAA_1e-3"))
    sub = full[full[:, 4] < 1e-4]
    key = lambda a: sorted(map(tuple, a[:, :2].astype(int)))  # noqa: E731
    assert key(allh) == key(sub)


def test_annotation_golden():
    bim = open(os.path.join(MOUSE_DATA, "plink.bim")).read().splitlines() if os.path.exists(
        os.path.join(MOUSE_DATA, "plink.bim")) else None
    if bim is None:
        pytest.skip("mouse data is only present in the build container")
    res = open(os.path.join(MOUSE_DATA, "epiAA_1e-3")).read().splitlines()
    got = O.annotation_snp_pos(res, bim, p_cut=1e-4, dis=1000000)
    exp = open(os.path.join(MOUSE_DATA, "epiAA_1e-3.anno")).read().splitlines()
    assert got == exp


def test_text_format_matches_reference():
    # rows written as the reference does (pandas to_csv of int, int, float64 repr)
    hdr, h = _load_hits(os.path.join(MOUSE_DATA, "epiAA_1e-5"))
    lines = open(os.path.join(MOUSE_DATA, "epiAA_1e-5")).read().splitlines()[1:]
    assert O.format_rows(h, 3) == lines


def test_tiny_text_outputs_md5():
    meta = json.load(open(os.path.join(TINY, "text_outputs.json")))
    ref = np.load(os.path.join(TINY, "tiny_ref.npz"))
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "k")
        np.savetxt(p, ref["agmat"])  # np.savetxt default '%.18e', as gmatrix.py:12
        assert hashlib.md5(open(p, "rb").read()).hexdigest() == meta[".agrm0"]["md5"]


def _eff_golden(name):
    lines = open(os.path.join(MOUSE_DATA, name)).read().splitlines()
    rows = [l.split() for l in lines[1:]]
    return lines[0], {(int(a[0]), int(a[1])): a[2:] for a in rows}


@pytest.fixture(scope="module")
def mouse_eff_inputs():
    prefix = os.path.join(MOUSE_DATA, "plink")
    snp = O.read_plink(prefix)
    n, m = snp.shape
    with open(prefix + ".bed", "rb") as f:
        dec = O.decode_bed(f.read(), n, m)
    a, d = O.agmat(snp), O.dgmat_as(snp)
    y, x, col, nid = O.design_matrix(os.path.join(MOUSE_DATA, "pheno"), prefix)
    ref = np.load(os.path.join(MOUSE_DATA, "reml.npz"))
    py2 = O.projection(y, x, col, nid, [a, a * a], ref["var2"])[1]
    py5 = O.projection(y, x, col, nid, [a, d, a * a, a * d, d * d], ref["var5"])[1]
    return dec, py2, py5


@pytest.mark.parametrize("kind,var_app", [("AA", 1470.0), ("AD", 960.0), ("DD", 490.0)])
def test_mouse_eff_screen_golden(mouse_eff_inputs, kind, var_app):
    """The C effect screen (_remma_epi_eff_cpu.c) and its chi_app / p_app post-processing
    (remma_epiAA_eff.py:85-95) on mouse rows 0..199 at a fixed threshold."""
    from scipy.stats import chi2
    dec, py2, py5 = mouse_eff_inputs
    cut = np.sqrt(chi2.isf(1e-2, 1) * var_app)
    got = O.epi_eff_screen(kind, dec, py2 if kind == "AA" else py5, range(200), cut)
    hdr, exp = _eff_golden("epi%s_eff_rows200" % kind)
    assert hdr == "snp_0 snp_1 eff chi_app p_app"
    got_d = {(int(i), int(j)): e for i, j, e in got}
    assert len(exp) > 1000
    near = {k for k, e in got_d.items() if abs(abs(e) - cut) < 1e-9 * cut}
    assert set(got_d) - near == set(exp) - near
    for k, cols in exp.items():
        assert abs(float(cols[0]) - got_d[k]) <= 5e-6 * abs(got_d[k]), (k, cols[0], got_d[k])
        chi_app = float(cols[0]) * float(cols[0]) / var_app
        assert cols[1] == repr(chi_app) and cols[2] == repr(float(chi2.sf(chi_app, 1)))


def _single_golden(path):
    lines = open(path).read().splitlines()
    assert lines[0] == "chro snp_ID pos allele1 allele2 eff_val chi_val eff_val_to_fixed p_val"
    vals = np.array([[float(v) if v else np.nan for v in (l.split(" ")[5:])] for l in lines[1:]])
    return lines, vals


@pytest.mark.parametrize("kind", ["add", "dom"])
def test_single_snp_golden(kind, tiny, mouse_eff_inputs):
    """remma_add / remma_dom restatement vs the reference's files (tiny: monomorphic SNPs give
    NaN statistics; the all-heterozygous SNP's dominance coding is a constant, so its numbers
    are rounding noise of an exact zero and only eff ~ 0 is checked)."""
    snp, ref, (y, x, col, nid) = tiny
    a, d = ref["agmat"], ref["dgmat"]
    g = [a, a * a] if kind == "add" else [a, d]
    pvp, py = O.projection(y, x, col, nid, g, ref["var"])
    sigma = ref["var"][0 if kind == "add" else 1]
    got = np.column_stack(O.remma_single(kind, snp, pvp, py, sigma))
    _, exp = _single_golden(os.path.join(TINY, "remma_" + kind))
    noise = np.abs(got[:, 0]) < 1e-12
    np.testing.assert_array_equal(np.isnan(got[~noise]), np.isnan(exp[~noise]))
    np.testing.assert_allclose(got[~noise], exp[~noise], rtol=1e-8, atol=1e-14)
    assert np.all(np.abs(exp[noise, 0]) < 1e-12)
    # mouse
    prefix = os.path.join(MOUSE_DATA, "plink")
    msnp = O.read_plink(prefix)
    ma, md = O.agmat(msnp), O.dgmat_as(msnp)
    my, mx, mcol, mnid = O.design_matrix(os.path.join(MOUSE_DATA, "pheno"), prefix)
    r = np.load(os.path.join(MOUSE_DATA, "reml.npz"))
    if kind == "add":
        pvp, py = O.projection(my, mx, mcol, mnid, [ma, ma * ma], r["var2"])
        sigma = r["var2"][0]
    else:
        pvp, py = O.projection(my, mx, mcol, mnid, [ma, md, ma * ma, ma * md, md * md], r["var5"])
        sigma = r["var5"][1]
    got = np.column_stack(O.remma_single(kind, msnp, pvp, py, sigma))
    _, exp = _single_golden(os.path.join(MOUSE_DATA, "remma_" + kind))
    np.testing.assert_allclose(got, exp, rtol=1e-8, atol=1e-14)


def test_repeated_records_golden(tiny):
    """Z != I: repeated, unordered records with a covariate (REML, exact AA scan) and the
    prediction workflow with record-less genotyped ids, against the reference's outputs."""
    _, ref, _ = tiny
    a = ref["agmat"]
    rep = np.load(os.path.join(TINY, "rep_ref.npz"))
    prefix = os.path.join(TINY, "tiny")
    y, x, col, nid = O.design_matrix(os.path.join(TINY, "rep.pheno"), prefix)
    assert y.shape[0] > nid and x.shape[1] == 2
    var = O.wemai_multi_gmat(y, x, col, nid, [a, a * a])
    np.testing.assert_allclose(var, rep["var"], rtol=1e-7)
    pvp, py = O.projection(y, x, col, nid, [a, a * a], rep["var"])
    snp = O.read_plink(prefix)
    got = O.epi_scan("AA", snp, pvp, py, p_cut=0.05)
    hdr, exp = _load_hits(os.path.join(TINY, "rep_epiAA"))
    assert got.shape == exp.shape
    np.testing.assert_array_equal(got[:, :2], exp[:, :2])
    np.testing.assert_allclose(got[:, 2:], exp[:, 2:], rtol=1e-8, atol=1e-300)
    y, x, col, nid = O.design_matrix_pred(os.path.join(TINY, "rep_pred.pheno"), prefix)
    assert nid == 150 and len(set(col.tolist())) == 135
    var = O.wemai_multi_gmat(y, x, col, nid, [a, a * a])
    np.testing.assert_allclose(var, rep["pred_var"], rtol=1e-7)
    re = O.predict_random(y, x, col, nid, [a, a * a], rep["pred_var"])
    np.testing.assert_allclose(re, rep["rand_eff"], rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("kind,base", [("AA", 1470.0), ("AD", 960.0), ("DD", 490.0)])
def test_mouse_maf_eff_screen_golden(mouse_eff_inputs, kind, base):
    """The per-class effect screens (print_out*_maf, _remma_epi_eff_cpu.c:141-166, :318-348,
    :500-522) and their post-processing (denominator of each written line from its own
    columns, remma_epiAD_maf_eff.py:102) with the classes of the _maf_approx pipelines."""
    from scipy.stats import chi2
    dec, py2, py5 = mouse_eff_inputs
    snp = O.read_plink(os.path.join(MOUSE_DATA, "plink"))
    fi, fj = O.maf_classes(kind, snp)
    deno = base * (0.8 + 0.004 * np.arange(111))
    cut = np.sqrt(chi2.isf(1e-2, 1) * deno)
    got = O.epi_eff_screen(kind, dec, py2 if kind == "AA" else py5, range(200), cut, freq_i=fi, freq_j=fj)
    hdr, exp = _eff_golden("epi%s_maf_eff_rows200" % kind)
    assert hdr == "snp_0 snp_1 eff chi_app p_app"
    got_d = {(int(i), int(j)): e for i, j, e in got}
    assert len(exp) > 1000 and set(got_d) == set(exp)
    for (i, j), cols in exp.items():
        assert abs(float(cols[0]) - got_d[(i, j)]) <= 5e-6 * abs(got_d[(i, j)])
        chi_app = float(float(cols[0]) * float(cols[0]) / deno[fi[i] * 10 + fj[j]])
        assert cols[1] == repr(chi_app) and cols[2] == repr(float(chi2.sf(chi_app, 1)))


README = os.path.join(os.path.dirname(__file__), "golden", "readme")


def test_readme_workflow_golden():
    """The README workflow fixture (missing calls, two covariates, seeded imputation, LD
    filter): the oracle's impute_geno with the same seed reproduces the reference's imputed
    GRM, its REML the variances, its scan the hit set, its annotation + LD filter the files."""
    prefix = os.path.join(README, "plink")
    snp = O.read_plink(prefix)
    assert np.isnan(snp).sum() > 0
    np.random.seed(1234)
    k = O.agmat(O.impute_geno(snp.copy()))
    ref_k = np.load(os.path.join(README, "agrm.npz"))["agrm"]
    np.testing.assert_allclose(k, ref_k, rtol=1e-12, atol=1e-14)
    y, x, col, nid = O.design_matrix(os.path.join(README, "pheno"), prefix)
    assert x.shape[1] == 3
    var = O.wemai_multi_gmat(y, x, col, nid, [ref_k, ref_k * ref_k])
    np.testing.assert_allclose(var, np.loadtxt(os.path.join(README, "var_a_axa.txt")), rtol=1e-8)
    np.random.seed(4321)
    snp2 = O.impute_geno(O.read_plink(prefix))
    var_ref = np.loadtxt(os.path.join(README, "var_a_axa.txt"))
    pvp, py = O.projection(y, x, col, nid, [ref_k, ref_k * ref_k], var_ref)
    exp = O.epi_scan("AA", snp2, pvp, py, p_cut=1e-2)
    got = np.loadtxt(os.path.join(README, "epiAA_a_axa"), skiprows=1, ndmin=2)
    np.testing.assert_array_equal(exp[:, :2], got[:, :2])
    np.testing.assert_allclose(exp[:, 2:], got[:, 2:], rtol=1e-9)
    res = open(os.path.join(README, "epiAA_a_axa")).read().splitlines()
    anno = O.annotation_snp_pos(res, open(prefix + ".bim").read().splitlines(), p_cut=1e-2, dis=0)
    assert [l.rstrip() for l in open(os.path.join(README, "epiAA_a_axa.anno")).read().splitlines()] == anno
    ld = O.ld_filter(anno, open(os.path.join(README, "plink.ld")).read().splitlines(), r2=0.2)
    exp_ld = open(os.path.join(README, "epiAA_a_axa.anno.ld")).read().splitlines()
    assert [l.rstrip() for l in exp_ld] == ld and len(ld) < len(anno)


REF_LIB = os.path.join(os.path.dirname(os.path.dirname(__file__)), "oracle", "_ref", "libremma_epi.so")


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="the reference's C is built only in the container")
@pytest.mark.parametrize("kind", ["AA", "AD", "DD"])
def test_eff_restatement_is_the_reference_bit_for_bit(kind, tmp_path):
    """oracle/eff_cpu.cpp against the reference's own _remma_epi_eff_cpu.c (compiled unmodified
    into oracle/_ref): identical record text ("%lld %lld %g") on a cohort with missing calls,
    duplicate and unsorted rows, single cut and _maf tables.  The reference runs single-threaded
    (its OpenMP loop interleaves rows nondeterministically)."""
    import subprocess
    import sys
    from gmat_amd import synth
    prefix = str(tmp_path / "c")
    n, m = 301, 420
    geno = synth.simulate_genotypes(n, m, seed=41, n_founder=20, n_gen=3, block=50)
    rng = np.random.default_rng(42)
    synth.write_plink(prefix, geno, missing=rng.random((m, n)) < 0.01, seed=41)
    py = rng.standard_normal(n)
    rows = np.array([3, 0, 77, 77, 250, m - 2, 11], dtype=np.int64)
    body = open(prefix + ".bed", "rb").read()[3:]
    fi = rng.integers(0, 11, m)
    fj = fi if kind != "AD" else rng.integers(0, 11, m)
    table = rng.uniform(0.5, 1.5, 111) * 8.0
    np.save(str(tmp_path / "py.npy"), py)
    np.save(str(tmp_path / "rows.npy"), rows)
    np.save(str(tmp_path / "fi.npy"), fi)
    np.save(str(tmp_path / "fj.npy"), fj)
    np.save(str(tmp_path / "table.npy"), table)
    script = """
import ctypes, numpy as np, sys
d, prefix, kind = sys.argv[1], sys.argv[2], sys.argv[3]
lib = ctypes.CDLL(%r)
py = np.load(d + '/py.npy'); rows = np.load(d + '/rows.npy'); fi = np.load(d + '/fi.npy'); fj = np.load(d + '/fj.npy')
table = np.load(d + '/table.npy')
P, L = ctypes.c_void_p, ctypes.c_longlong
n, m = %d, %d
f = getattr(lib, 'remma_epi%%s_eff_cpu' %% kind)
f.argtypes = [ctypes.c_char_p, L, L, P, L, P, ctypes.c_double, ctypes.c_char_p]
f(prefix.encode(), n, m, rows.ctypes.data, rows.size, py.ctypes.data, 8.0, (d + '/ref_single').encode())
g = getattr(lib, 'remma_epi%%s_maf_eff_cpu' %% kind)
if kind == 'AD':
    g.argtypes = [ctypes.c_char_p, L, L, P, L, P, P, P, P, ctypes.c_char_p]
    g(prefix.encode(), n, m, rows.ctypes.data, rows.size, py.ctypes.data, fi.ctypes.data, fj.ctypes.data,
      table.ctypes.data, (d + '/ref_maf').encode())
else:
    g.argtypes = [ctypes.c_char_p, L, L, P, L, P, P, P, ctypes.c_char_p]
    g(prefix.encode(), n, m, rows.ctypes.data, rows.size, py.ctypes.data, fi.ctypes.data, table.ctypes.data,
      (d + '/ref_maf').encode())
""" % (REF_LIB, n, m)
    env = dict(os.environ, OMP_NUM_THREADS="1")
    subprocess.run([sys.executable, "-c", script, str(tmp_path), prefix, kind], check=True, env=env,
                   stdout=subprocess.DEVNULL)
    for name, cut, a, b in (("ref_single", [8.0], None, None), ("ref_maf", table, fi, fj)):
        i, j, e = O.eff_screen_c(kind, body, n, m, rows, py, cut, a, b)
        text = "snp_0 snp_1 eff\n" + "".join("%d %d %s\n" % (u, v, "%g" % w) for u, v, w in zip(i, j, e))
        assert i.size > 20
        assert open(str(tmp_path / name)).read() == text
