"""The pair screen (pair_side_kernel + pair_mx_kernel: every screen candidate re-tested with the MX
quadratic form and exact fp64 side terms before the refine) drops only pairs whose p-value is
certainly >= p_cut: hits with it are identical to hits without it (GMAT_NO_PAIR_SCREEN) and to the
oracle's (remma_epiAA.py:71-82 and siblings), for every kind and screen level, at p_cut values
from a thin candidate band to one where most candidates are hits."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cohort(tmp_path_factory):
    from gmat_amd import synth
    from oracle import gmat_oracle as O
    d = tmp_path_factory.mktemp("ps")
    prefix = os.path.join(str(d), "c")
    synth.make_cohort(prefix, 640, 2600, seed=23)
    snp = O.read_plink(prefix)
    ka = O.agmat(snp)
    y, x, col, nid = O.design_matrix(prefix + ".pheno", prefix)
    pvp, py = O.projection(y, x, col, nid, [ka, ka * ka], np.array([0.4, 0.2, 0.4]))
    return prefix, snp, pvp, py


def _scan(plan, kind, rows, p_cut, level, off):
    if off:
        os.environ["GMAT_NO_PAIR_SCREEN"] = "1"
    try:
        return plan.scan(kind, rows, p_cut, n_slice=level)
    finally:
        os.environ.pop("GMAT_NO_PAIR_SCREEN", None)


@pytest.mark.parametrize("kind", ["AA", "AD", "DD"])
def test_pair_screen_keeps_every_hit(cohort, kind):
    from gmat_amd.plink import Geno
    from gmat_amd.remma._scan import EpiPlan
    from oracle import gmat_oracle as O
    prefix, snp, pvp, py = cohort
    rows = np.array([0, 5, 640, 1301, 2050, 2598])
    with Geno(prefix) as g, EpiPlan(g, pvp, py[:, 0]) as plan:
        levels = (-2, -1, 0, 2) if plan.lowrank_rank() > 0 else (-1, 0, 2)
        for p_cut in (1e-3, 2e-2, 0.2):
            exp = O.epi_scan(kind, snp, pvp, py, snp_lst_0=rows, p_cut=p_cut)
            for level in levels:
                a = _scan(plan, kind, rows, p_cut, level, off=False)
                b = _scan(plan, kind, rows, p_cut, level, off=True)
                for u, v in zip(a, b):
                    np.testing.assert_array_equal(u, v)
                np.testing.assert_array_equal(a[0], exp[:, 0].astype(np.int64))
                np.testing.assert_array_equal(a[1], exp[:, 1].astype(np.int64))
                np.testing.assert_allclose(a[5], exp[:, 4], rtol=1e-8)


@pytest.fixture(scope="module")
def wide_cohort(tmp_path_factory):
    """n_pad 2,176 (17 stages of 128): past the 16 stages a wave holds, so the pair screen runs by squares
    of stages (pair_mxw_kernel: segments 16 x 16, 16 x 1 and 1 x 1)."""
    from gmat_amd import synth
    from oracle import gmat_oracle as O
    d = tmp_path_factory.mktemp("psw")
    prefix = os.path.join(str(d), "c")
    synth.make_cohort(prefix, 2100, 1500, seed=29)
    snp = O.read_plink(prefix)
    ka = O.agmat(snp)
    y, x, col, nid = O.design_matrix(prefix + ".pheno", prefix)
    pvp, py = O.projection(y, x, col, nid, [ka, ka * ka], np.array([0.4, 0.2, 0.4]))
    return prefix, snp, pvp, py


@pytest.mark.parametrize("kind", ["AA", "AD"])
def test_pair_screen_by_stage_squares_keeps_every_hit(wide_cohort, kind):
    from gmat_amd.plink import Geno
    from gmat_amd.remma._scan import EpiPlan
    from oracle import gmat_oracle as O
    prefix, snp, pvp, py = wide_cohort
    rows = np.array([0, 7, 733, 1498])
    with Geno(prefix) as g, EpiPlan(g, pvp, py[:, 0]) as plan:
        for p_cut in (1e-3, 2e-2):
            exp = O.epi_scan(kind, snp, pvp, py, snp_lst_0=rows, p_cut=p_cut)
            for level in ((-1, 0) if plan.lowrank_rank() > 0 else (0,)):
                a = _scan(plan, kind, rows, p_cut, level, off=False)
                b = _scan(plan, kind, rows, p_cut, level, off=True)
                for u, v in zip(a, b):
                    np.testing.assert_array_equal(u, v)
                np.testing.assert_array_equal(a[0], exp[:, 0].astype(np.int64))
                np.testing.assert_array_equal(a[1], exp[:, 1].astype(np.int64))
                np.testing.assert_allclose(a[5], exp[:, 4], rtol=1e-8)
