"""Hit decisions at the threshold: pairs placed at
p = p_cut (1 +- 1e-10) are kept / dropped exactly as the oracle's fp64 computation decides
(remma_epiAA.py:71-82: p = chi2.sf(chi, 1) < p_cut), at every screen level.

The device computes p = erfc(sqrt(chi / 2)) (the same function as chi2.sf for one degree of
freedom); the reference goes through cephes igamc.  Both are accurate to a few ulps, so a
relative margin of 1e-10 separates the decision from either rounding: the symmetric difference
of the hit sets must be empty.  Pairs closer to the threshold than ~1e-15 relative are the only
ones whose decision can depend on the library, and no test here places one there."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cohort(tmp_path_factory):
    from gmat_amd import synth
    from oracle import gmat_oracle as O
    d = tmp_path_factory.mktemp("thr")
    prefix = os.path.join(str(d), "c")
    synth.make_cohort(prefix, 600, 3000, seed=11)
    snp = O.read_plink(prefix)
    ka = O.agmat(snp)
    y, x, col, nid = O.design_matrix(prefix + ".pheno", prefix)
    pvp, py = O.projection(y, x, col, nid, [ka, ka * ka], np.array([0.4, 0.2, 0.4]))
    rows = np.array([0, 3, 777, 1500, 2222, 2997])
    exp = O.epi_scan("AA", snp, pvp, py, snp_lst_0=rows, p_cut=2e-2)
    return prefix, snp, pvp, py, rows, exp


@pytest.mark.parametrize("level", [0, -2, -1, 1])
def test_pairs_at_the_threshold(cohort, level):
    from gmat_amd.plink import Geno
    from gmat_amd.remma._scan import EpiPlan
    prefix, snp, pvp, py, rows, exp = cohort
    order = np.argsort(exp[:, 4])
    targets = exp[order[np.linspace(0, len(order) - 1, 8).astype(int)]]  # smallest p to ~2e-2
    assert targets.shape[0] == 8 and targets[0, 4] < 1e-3
    with Geno(prefix) as g, EpiPlan(g, pvp, py[:, 0]) as plan:
        for i, j, _, _, pk in targets:
            for rel, inside in ((1.0 + 1e-10, True), (1.0 - 1e-10, False)):
                p_cut = pk * rel
                hi, hj, eff, var, chi, p = plan.scan("AA", rows, p_cut, n_slice=level)
                want = exp[exp[:, 4] < p_cut]
                got = set(zip(hi.tolist(), hj.tolist()))
                ref = set(zip(want[:, 0].astype(int).tolist(), want[:, 1].astype(int).tolist()))
                assert got == ref, (level, p_cut, sorted(got ^ ref)[:5])
                assert ((int(i), int(j)) in got) == inside
                np.testing.assert_allclose(p, want[:, 4], rtol=1e-10)
