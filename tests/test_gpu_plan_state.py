"""A plan's spectral state (eigendecomposition, prefilter and low-rank certificates, the low-rank
basis' tile images) exported by one plan and imported by another (gmat_epi_export /
gmat_epi_create_with: what dist.shared_plan broadcasts from rank 0): the importing plan skips the
eigendecomposition and certificate searches and scans exactly as the exporting plan does."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cohort(tmp_path_factory):
    from gmat_amd import synth
    from oracle import gmat_oracle as O
    from scipy.sparse import identity
    from gmat_amd.uvlmm.uvlmm_varcom import projection
    d = tmp_path_factory.mktemp("state")
    prefix = os.path.join(str(d), "c")
    synth.make_cohort(prefix, 700, 2500, seed=5)
    snp = O.read_plink(prefix)
    ka = O.agmat(snp)
    rng = np.random.default_rng(3)
    n = snp.shape[0]
    y = 1.0 + rng.standard_normal(n)
    x1 = np.ones((n, 1))
    x3 = np.column_stack([np.ones(n), rng.integers(0, 2, n), rng.integers(90, 130, n)]).astype(float)
    ps = [projection(y, x, identity(n, format="csr"), [ka, ka * ka], [0.4, 0.2, 0.4]) for x in (x1, x3)]
    return prefix, ps


@pytest.mark.parametrize("design", [0, 1])
def test_imported_state_scans_identically(cohort, design):
    from gmat_amd import _native as N
    from gmat_amd.plink import Geno
    from gmat_amd.remma._scan import EpiPlan
    prefix, ps = cohort
    pvp, py = ps[design]
    rows = np.array([0, 1, 600, 1249, 2400, 2498])
    with Geno(prefix) as g:
        with EpiPlan(g, pvp, py) as a:
            st = a.export_state()
            assert st.size > 64
            sa = a.setup_stats()
            with EpiPlan(g, pvp, py, state=st) as b:
                sb = b.setup_stats()
                assert sb["eigen_s"] == 0.0 and sb["cholesky_count"] == 0.0, sb
                assert sb["covariate_directions"] == sa["covariate_directions"] == 2 * design
                assert b.lowrank_rank() == a.lowrank_rank() > 0
                np.testing.assert_array_equal(b.export_state(), st)
                for kind, p_cut, level in (("AA", 1e-3, -2), ("AA", 1e-2, -1), ("DD", 1e-2, 0), ("AD", 1e-3, -2)):
                    ra = a.scan(kind, rows, p_cut, n_slice=level)
                    rb = b.scan(kind, rows, p_cut, n_slice=level)
                    assert ra[0].size > 0
                    for u, v in zip(ra, rb):
                        np.testing.assert_array_equal(u, v)
        other = ps[1 - design][0]
        with pytest.raises(N.GmatNativeError, match="different P"):
            EpiPlan(g, other, py, state=st)
        with pytest.raises(N.GmatNativeError):
            EpiPlan(g, pvp, py, state=st[:-8])
