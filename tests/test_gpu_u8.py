"""U = codes x P (the codings' side vectors) on int8 slices of P (u8_gemm_kernel in csrc/epi_*.hip)
against the fp64 GEMM it replaced (GMAT_U_DGEMM=1): the scan's hits and statistics and the exact
refine of sampled pairs agree to fp64 rounding (the slicing error is bounded below 2^-46 of a row's
largest |P|), and the default path is checked against the oracle (remma_epiAA.py:71-82)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cohort(tmp_path_factory):
    from gmat_amd import synth
    from oracle import gmat_oracle as O
    d = tmp_path_factory.mktemp("u8")
    prefix = os.path.join(str(d), "c")
    synth.make_cohort(prefix, 650, 2700, seed=7)  # m not a multiple of the 256-SNP workgroup tile
    snp = O.read_plink(prefix)
    ka = O.agmat(snp)
    y, x, col, nid = O.design_matrix(prefix + ".pheno", prefix)
    pvp, py = O.projection(y, x, col, nid, [ka, ka * ka], np.array([0.4, 0.2, 0.4]))
    return prefix, snp, pvp, py


def _run(prefix, pvp, py, kind, rows, pairs, dgemm):
    from gmat_amd.plink import Geno
    from gmat_amd.remma._scan import EpiPlan
    old = os.environ.pop("GMAT_U_DGEMM", None)
    if dgemm:
        os.environ["GMAT_U_DGEMM"] = "1"
    try:
        with Geno(prefix) as g, EpiPlan(g, pvp, py[:, 0]) as plan:
            hits = plan.scan(kind, rows, 1e-4)  # the codings (and U) are built here
            exact = plan.pairs(kind, pairs)
    finally:
        os.environ.pop("GMAT_U_DGEMM", None)
        if old is not None:
            os.environ["GMAT_U_DGEMM"] = old
    return hits, exact


@pytest.mark.parametrize("kind", ["AA", "AD", "DD"])
def test_int8_slice_u_matches_fp64_gemm(cohort, kind):
    from oracle import gmat_oracle as O
    prefix, snp, pvp, py = cohort
    m = snp.shape[1]
    rows = np.arange(m - 1 if kind != "AD" else m, dtype=np.int64)
    rng = np.random.default_rng(3)
    pairs = np.sort(rng.integers(0, m, size=(3000, 2)), axis=1)
    pairs = pairs[pairs[:, 0] < pairs[:, 1]]
    h8, e8 = _run(prefix, pvp, py, kind, rows, pairs, dgemm=False)
    h64, e64 = _run(prefix, pvp, py, kind, rows, pairs, dgemm=True)
    assert h8[0].size > 20
    np.testing.assert_array_equal(h8[0], h64[0])
    np.testing.assert_array_equal(h8[1], h64[1])
    for a, b in zip(h8[2:], h64[2:]):
        np.testing.assert_allclose(a, b, rtol=1e-11, atol=0)
    for a, b in zip(e8[:2], e64[:2]):  # eff (no U), var
        np.testing.assert_allclose(a, b, rtol=1e-11, atol=1e-300)
    # the default path against the oracle on sampled rows
    sample = np.array([0, 5, 999, 2100, m - 2])
    exp = O.epi_scan(kind, snp, pvp, py, snp_lst_0=sample, p_cut=1e-4)
    sel = np.isin(h8[0], sample)
    np.testing.assert_array_equal(h8[0][sel], exp[:, 0].astype(np.int64))
    np.testing.assert_array_equal(h8[1][sel], exp[:, 1].astype(np.int64))
    np.testing.assert_allclose(h8[5][sel], exp[:, 4], rtol=1e-8)
