"""Parity of the GPU effect screen and the approximate pipelines.

* the drop-in C symbols remma_epi{AA,AD,DD}(_maf)_eff_cpu and read_plink_bed, called through
  ctypes with the reference's prototypes, against the oracle's restatement of
  _remma_epi_eff_cpu.c on a cohort with missing calls (coded 1/3, as the C code decodes them);
* the Python pipelines remma_epiXX_eff against the golden files the reference wrote on mouse;
* remma_epiXX_approx / _maf_approx end to end against the oracle (seeded random pairs).

Bars: the kept pair sets are identical except pairs within 1e-9 relative of the threshold
(none occur in these data); eff within 1e-9 relative of the oracle (5e-6 against the
reference's 6-digit %g text); the chi_app / p_app text is the reference's formula applied to
the written eff.
"""
import os
import shutil

import numpy as np
import pytest
from scipy.stats import chi2

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
MOUSE = os.path.join(GOLD, "mouse")


def _read_eff(path):
    lines = open(path).read().splitlines()
    return lines[0], [l.split() for l in lines[1:]]


def _check_vs_oracle(path, exp, cut_of):
    """File rows vs the oracle's sorted (i, j, eff) list; cut_of(i, j) -> threshold."""
    hdr, rows = _read_eff(path)
    assert hdr == "snp_0 snp_1 eff"
    got = {(int(a[0]), int(a[1])): float(a[2]) for a in rows}  # duplicate list rows repeat lines
    want = {(int(i), int(j)): e for i, j, e in exp}
    near = {k for k, e in want.items() if abs(abs(e) - cut_of(*k)) < 1e-9 * cut_of(*k)}
    assert set(got) - near == set(want) - near
    for k in got:
        if k in want:
            assert float("%g" % want[k]) == pytest.approx(got[k], rel=1e-9), k
    return rows


@pytest.fixture(scope="module")
def cohort(tmp_path_factory):
    """350 x 700 related cohort with ~0.5 % missing calls (2-bit code 01)."""
    from gmat_amd import synth
    d = tmp_path_factory.mktemp("effc")
    prefix = os.path.join(str(d), "c")
    synth.make_cohort(prefix, 350, 700, seed=21)
    raw = bytearray(open(prefix + ".bed", "rb").read())
    rng = np.random.default_rng(5)
    n, m = 350, 700
    nb = (n + 3) // 4
    for j, k in zip(rng.integers(0, m, 1200), rng.integers(0, n, 1200)):
        off = 3 + j * nb + k // 4
        sh = 2 * (k % 4)
        raw[off] = (raw[off] & ~(3 << sh) & 0xFF) | (1 << sh)
    open(prefix + ".bed", "wb").write(bytes(raw))
    from oracle import gmat_oracle as O
    dec = O.decode_bed(bytes(raw), n, m)
    py = rng.standard_normal(n)
    return prefix, dec, py


def test_read_plink_bed_symbol(cohort):
    from gmat_amd import _native as N
    prefix, dec, _ = cohort
    lib = N.ensure_device()
    m, n = dec.shape
    out = np.zeros((m, n))
    assert lib.read_plink_bed(prefix.encode(), n, m, N.ptr(out)) == 1
    np.testing.assert_array_equal(out, dec)
    # missing file / bad magic: an error code, not exit()
    assert lib.read_plink_bed(b"/nonexistent/x", n, m, N.ptr(out)) < 0


@pytest.mark.parametrize("kind", ["AA", "AD", "DD"])
def test_eff_symbols_vs_oracle(cohort, kind, tmp_path):
    from oracle import gmat_oracle as O
    from gmat_amd import _native as N
    prefix, dec, py = cohort
    lib = N.ensure_device()
    m, n = dec.shape
    top = m if kind == "AD" else m - 1
    rows = np.array([5, 0, 17, 17, 311, top - 1, 698 if kind != "AD" else 699, 2, 640], dtype=np.longlong)
    # threshold at the 90th percentile of |eff| of row 0
    probe = O.epi_eff_screen(kind, dec, py, [0], 0.0)
    cut = float(np.quantile([abs(e) for _, _, e in probe], 0.9))
    out = str(tmp_path / "eff")
    sym = getattr(lib, "remma_epi%s_eff_cpu" % kind)
    assert sym(prefix.encode(), n, m, N.ptr(rows), rows.size, N.ptr(py), cut, out.encode()) == 1
    exp, order = [], []
    for r in rows.tolist():  # list order, duplicates kept
        part = O.epi_eff_screen(kind, dec, py, [r], cut)
        exp += part
        # the reference's single-thread order: j ascending, AD (i, j) before (j, i)
        part.sort(key=lambda t: (t[1], 0) if t[0] == r else (t[0], 1))
        order += [(int(i), int(j)) for i, j, _ in part]
    got_rows = _check_vs_oracle(out, exp, lambda i, j: cut)
    assert [(int(a[0]), int(a[1])) for a in got_rows] == order
    # empty list -> header only
    assert sym(prefix.encode(), n, m, N.ptr(rows), 0, N.ptr(py), cut, out.encode()) == 1
    assert open(out).read() == "snp_0 snp_1 eff\n"

    # the _maf form: per-class thresholds, class arrays 0..10
    rng = np.random.default_rng(3)
    fi = rng.integers(0, 11, m).astype(np.longlong)
    fj = fi if kind != "AD" else rng.integers(0, 11, m).astype(np.longlong)
    table = np.ascontiguousarray(cut * rng.uniform(0.7, 1.3, 111))
    msym = getattr(lib, "remma_epi%s_maf_eff_cpu" % kind)
    if kind == "AD":
        rc = msym(prefix.encode(), n, m, N.ptr(rows), rows.size, N.ptr(py), N.ptr(fi), N.ptr(fj), N.ptr(table),
                  out.encode())
    else:
        rc = msym(prefix.encode(), n, m, N.ptr(rows), rows.size, N.ptr(py), N.ptr(fi), N.ptr(table), out.encode())
    assert rc == 1
    exp = []
    for r in rows.tolist():
        exp += O.epi_eff_screen(kind, dec, py, [r], table, freq_i=fi, freq_j=fj)
    # the threshold of a written (j, i) AD line is the (i, j) class pair
    cut_of = (lambda i, j: table[fi[min(i, j)] * 10 + fj[max(i, j)]]) if kind == "AD" else \
        (lambda i, j: table[fi[i] * 10 + fj[j]])
    _check_vs_oracle(out, exp, cut_of)
    # out-of-range class -> error, no crash
    bad = fi.copy()
    bad[3] = 11
    if kind == "AD":
        rc = msym(prefix.encode(), n, m, N.ptr(rows), rows.size, N.ptr(py), N.ptr(bad), N.ptr(fj), N.ptr(table),
                  out.encode())
    else:
        rc = msym(prefix.encode(), n, m, N.ptr(rows), rows.size, N.ptr(py), N.ptr(bad), N.ptr(table), out.encode())
    assert rc < 0


@pytest.mark.parametrize("kind", ["AA", "AD", "DD"])
def test_eff_symbols_bit_identical_to_restatement(cohort, kind, tmp_path):
    """The GPU screen + exact recompute reproduce the reference's fp64 arithmetic: the written
    file equals, byte for byte, the C++ restatement's (oracle/eff_cpu.cpp, itself checked
    bit-for-bit against the reference's own C in the container), single cut and _maf table."""
    from oracle import gmat_oracle as O
    from gmat_amd import _native as N
    prefix, dec, py = cohort
    lib = N.ensure_device()
    m, n = dec.shape
    body = open(prefix + ".bed", "rb").read()[3:]
    rows = np.array([9, 0, 400, 400, 13, m - 2, 250], dtype=np.longlong)
    probe = O.epi_eff_screen(kind, dec, py, [0], 0.0)
    cut = float(np.quantile([abs(e) for _, _, e in probe], 0.8))
    out = str(tmp_path / "eff")
    assert getattr(lib, "remma_epi%s_eff_cpu" % kind)(prefix.encode(), n, m, N.ptr(rows), rows.size, N.ptr(py), cut,
                                                      out.encode()) == 1
    i, j, e = O.eff_screen_c(kind, body, n, m, rows, py, [cut])
    assert i.size > 100
    assert open(out).read() == "snp_0 snp_1 eff\n" + "".join("%d %d %s\n" % (u, v, "%g" % w) for u, v, w in zip(i, j, e))
    rng = np.random.default_rng(8)
    fi = rng.integers(0, 11, m).astype(np.longlong)
    fj = fi if kind != "AD" else rng.integers(0, 11, m).astype(np.longlong)
    table = np.ascontiguousarray(cut * rng.uniform(0.6, 1.4, 111))
    msym = getattr(lib, "remma_epi%s_maf_eff_cpu" % kind)
    args = (N.ptr(fi), N.ptr(fj)) if kind == "AD" else (N.ptr(fi),)
    assert msym(prefix.encode(), n, m, N.ptr(rows), rows.size, N.ptr(py), *args, N.ptr(table), out.encode()) == 1
    i, j, e = O.eff_screen_c(kind, body, n, m, rows, py, table, fi, fj)
    assert open(out).read() == "snp_0 snp_1 eff\n" + "".join("%d %d %s\n" % (u, v, "%g" % w) for u, v, w in zip(i, j, e))


@pytest.fixture(scope="module")
def mouse(tmp_path_factory):
    d = tmp_path_factory.mktemp("mouse_eff")
    for f in ("plink.bed", "plink.bim", "plink.fam", "pheno"):
        shutil.copy(os.path.join(MOUSE, f), str(d))
    prefix = os.path.join(str(d), "plink")
    from gmat_amd.gmatrix import agmat, dgmat_as
    ka, _ = agmat(prefix)
    kd, _ = dgmat_as(prefix)
    ref = np.load(os.path.join(MOUSE, "reml.npz"))
    return prefix, [ka, ka * ka], [ka, kd, ka * ka, ka * kd, kd * kd], ref["var2"], ref["var5"]


@pytest.mark.parametrize("kind,var_app", [("AA", 1470.0), ("AD", 960.0), ("DD", 490.0)])
def test_mouse_eff_golden(mouse, kind, var_app, tmp_path):
    """remma_epiXX_eff on mouse rows 0..199 against the file the reference wrote."""
    import importlib
    prefix, g2, g5, var2, var5 = mouse
    fn = getattr(importlib.import_module("gmat_amd.remma.remma_epi%s" % kind), "remma_epi%s_eff" % kind)
    g, var = (g2, var2) if kind == "AA" else (g5, var5)
    out = str(tmp_path / kind)
    assert fn(prefix.replace("plink", "pheno"), prefix, g, var, snp_lst_0=list(range(200)), var_app=var_app,
              p_cut=1e-2, out_file=out) == 0
    assert not os.path.exists(out + ".temp")
    hdr, got = _read_eff(out)
    ehdr, exp = _read_eff(os.path.join(MOUSE, "epi%s_eff_rows200" % kind))
    assert hdr == ehdr == "snp_0 snp_1 eff chi_app p_app"
    gd = {(a[0], a[1]): a[2:] for a in got}
    ed = {(a[0], a[1]): a[2:] for a in exp}
    assert set(gd) == set(ed)
    same_text = 0
    for k, cols in gd.items():
        assert float(cols[0]) == pytest.approx(float(ed[k][0]), rel=5e-6)
        same_text += cols[0] == ed[k][0]
        chi_app = float(cols[0]) * float(cols[0]) / var_app
        assert cols[1] == repr(chi_app) and cols[2] == repr(float(chi2.sf(chi_app, 1)))
    assert same_text >= 0.99 * len(gd)


def _oracle_setup(prefix, gmats_kind):
    from oracle import gmat_oracle as O
    snp = O.read_plink(prefix)
    n, m = snp.shape
    with open(prefix + ".bed", "rb") as f:
        dec = O.decode_bed(f.read(), n, m)
    a, d = O.agmat(snp), O.dgmat_as(snp)
    y, x, col, nid = O.design_matrix(prefix.replace("plink", "pheno"), prefix)
    ref = np.load(os.path.join(MOUSE, "reml.npz"))
    if gmats_kind == "AA":
        pvp, py = O.projection(y, x, col, nid, [a, a * a], ref["var2"])
    else:
        pvp, py = O.projection(y, x, col, nid, [a, d, a * a, a * d, d * d], ref["var5"])
    return O, snp, dec, pvp, py


@pytest.mark.parametrize("kind,maf", [("AA", False), ("AD", False), ("DD", False), ("AA", True), ("DD", True), ("AD", True)])
def test_mouse_approx_pipeline(mouse, kind, maf, tmp_path):
    """remma_epiXX_approx / _maf_approx with seeded random pairs, end to end vs the oracle:
    variance estimate from the same random pairs, screen survivors, exact re-test, merge."""
    import importlib
    from gmat_amd.remma.random_pair import random_pair, random_pairAD
    prefix, g2, g5, var2, var5 = mouse
    g, var = (g2, var2) if kind == "AA" else (g5, var5)
    mod = importlib.import_module("gmat_amd.remma.remma_epi%s" % kind)
    name = "remma_epi%s_%sapprox" % (kind, "maf_" if maf else "")
    out = str(tmp_path / name)
    cwd = os.getcwd()
    os.chdir(str(tmp_path))
    try:
        assert getattr(mod, name)(prefix.replace("plink", "pheno"), prefix, g, var, p_cut=1e-3,
                                  num_random_pair=6000, out_file=out, seed=11) == 0
    finally:
        os.chdir(cwd)
    O, snp, dec, pvp, py = _oracle_setup(prefix, kind)
    m = dec.shape[0]
    pairs = (random_pairAD if kind == "AD" else random_pair)(m, out_file=str(tmp_path / "rp"), num_pair=6000,
                                                              seed=11)
    _, rv, _, _ = O.epi_pair(kind, snp, pvp, py, pairs)
    rows = range(m) if kind == "AD" else range(m - 1)
    if maf:
        fi, fj = O.maf_classes(kind, snp)
        deno = O.class_denominators(kind, list(zip(pairs[:, 0].tolist(), pairs[:, 1].tolist(), rv.tolist())), fi, fj)
        exp = O.epi_eff_screen(kind, dec, py, rows, np.sqrt(chi2.isf(1e-3, 1) * deno), freq_i=fi, freq_j=fj)
        den_of = lambda i, j: deno[fi[i] * 10 + fj[j]]  # noqa: E731  (post-processing: line's own columns)
    else:
        vmed = np.median(rv)
        exp = O.epi_eff_screen(kind, dec, py, rows, np.sqrt(chi2.isf(1e-3, 1) * vmed))
        den_of = lambda i, j: vmed  # noqa: E731
    lines = open(out).read().splitlines()
    assert lines[0] == "snp_0 snp_1 eff var chi p_app p"
    got = [l.split() for l in lines[1:]]
    assert len(exp) > 5
    assert sorted((int(a[0]), int(a[1])) for a in got) == sorted((int(i), int(j)) for i, j, _ in exp)
    gp = np.array([[int(a[0]), int(a[1])] for a in got], dtype=np.int64)
    eff, var_, chi_, p = O.epi_pair(kind, snp, pvp, py, gp)
    vals = np.array([[float(v) for v in a[2:5] + a[6:7]] for a in got])
    np.testing.assert_allclose(vals, np.column_stack([eff, var_, chi_, p]), rtol=1e-8)
    ed = {(int(i), int(j)): e for i, j, e in exp}
    for a in got:
        e_txt = float("%g" % ed[(int(a[0]), int(a[1]))])
        p_app = chi2.sf(e_txt * e_txt / den_of(int(a[0]), int(a[1])), 1)
        assert float(a[5]) == pytest.approx(float(p_app), rel=1e-9)


def _single(path):
    lines = open(path).read().splitlines()
    vals = np.array([[float(v) if v else np.nan for v in l.split(" ")[5:]] for l in lines[1:]])
    return lines, vals


@pytest.mark.parametrize("kind", ["add", "dom"])
def test_single_snp_golden(mouse, kind, tmp_path):
    """remma_add / remma_dom against the reference's files on mouse and
    tiny (monomorphic SNPs: eff 0.0 and empty NaN fields; the all-heterozygous SNP of the
    dominance test is rounding noise of an exact zero in the reference and is only checked
    for eff ~ 0)."""
    import gmat_amd.remma as R
    fn = R.remma_add if kind == "add" else R.remma_dom
    prefix, g2, g5, var2, var5 = mouse
    out = str(tmp_path / "m")
    df = fn(prefix.replace("plink", "pheno"), prefix, g2 if kind == "add" else g5, var2 if kind == "add" else var5,
            out_file=out)
    gl, gv = _single(out)
    el, ev = _single(os.path.join(MOUSE, "remma_" + kind))
    assert len(gl) == len(el) and gl[0] == el[0]
    assert [l.split(" ")[:5] for l in gl] == [l.split(" ")[:5] for l in el]
    np.testing.assert_allclose(gv, ev, rtol=1e-8, atol=1e-14)
    assert df.shape == (len(gl) - 1, 9)
    # tiny
    d = tmp_path / "tiny"
    d.mkdir()
    for ext in (".bed", ".bim", ".fam", ".pheno"):
        shutil.copy(os.path.join(GOLD, "tiny", "tiny" + ext), str(d))
    tp = str(d / "tiny")
    ref = np.load(os.path.join(GOLD, "tiny", "tiny_ref.npz"))
    a, dm = ref["agmat"], ref["dgmat"]
    fn(tp + ".pheno", tp, [a, a * a] if kind == "add" else [a, dm], ref["var"], out_file=tp + ".out")
    gl, gv = _single(tp + ".out")
    el, ev = _single(os.path.join(GOLD, "tiny", "remma_" + kind))
    assert [l.split(" ")[:5] for l in gl] == [l.split(" ")[:5] for l in el]
    noise = np.abs(ev[:, 0]) < 1e-12
    assert np.all(np.abs(gv[noise, 0]) < 1e-12)
    np.testing.assert_array_equal(np.isnan(gv[~noise]), np.isnan(ev[~noise]))
    np.testing.assert_allclose(gv[~noise], ev[~noise], rtol=1e-8, atol=1e-14)


@pytest.mark.parametrize("kind,base", [("AA", 1470.0), ("AD", 960.0), ("DD", 490.0)])
def test_mouse_maf_eff_golden(mouse, kind, base, tmp_path):
    """remma_epiXX_maf_eff (per-class thresholds) on mouse rows 0..199 against the reference's
    files: same pair sets, eff %g text, chi_app / p_app from each line's own classes."""
    import importlib
    from oracle import gmat_oracle as O
    prefix, g2, g5, var2, var5 = mouse
    fi, fj = O.maf_classes(kind, O.read_plink(prefix))
    deno = base * (0.8 + 0.004 * np.arange(111))
    mod = importlib.import_module("gmat_amd.remma.remma_epi%s" % kind)
    fn = getattr(mod, "remma_epi%s_maf_eff" % kind)
    out = str(tmp_path / kind)
    kw = dict(freqA=fi, freqD=fj) if kind == "AD" else dict(freq=fi)
    cwd = os.getcwd()
    os.chdir(str(tmp_path))
    try:
        assert fn(prefix.replace("plink", "pheno"), prefix, g2 if kind == "AA" else g5, var2 if kind == "AA" else var5,
                  snp_lst_0=list(range(200)), freq_deno=deno, p_cut=1e-2, out_file=out, **kw) == 0
    finally:
        os.chdir(cwd)
    if kind != "AD":
        assert os.path.exists(str(tmp_path / "eff_cut"))  # written to the working directory, as the reference
    hdr, got = _read_eff(out)
    ehdr, exp = _read_eff(os.path.join(MOUSE, "epi%s_maf_eff_rows200" % kind))
    assert hdr == ehdr
    gd = {(a[0], a[1]): a[2:] for a in got}
    ed = {(a[0], a[1]): a[2:] for a in exp}
    assert set(gd) == set(ed) and len(gd) > 1000
    same = 0
    for k, cols in gd.items():
        assert float(cols[0]) == pytest.approx(float(ed[k][0]), rel=5e-6)
        same += cols == ed[k]
    assert same >= 0.99 * len(gd)
