"""The scan plan's partial symmetric eigensolver (gmat_amd/csrc/eig.hip) against numpy's dense
decomposition, on projection matrices P of the kind the plan decomposes (uvlmm_varcom.py:
P = V^-1 - V^-1 X (X'V^-1 X)^-1 X'V^-1, intercept direction lifted as epi.hip eigen_bottom does),
with and without covariates (P's exact null directions: a repeated eigenvalue 0)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _p_matrix(n, m, ncov, seed):
    rng = np.random.default_rng(seed)
    # a related cohort: founders' haplotype blocks shared by families of 4
    base = rng.integers(0, 3, size=(n // 4 + 1, m)).astype(float)
    g = np.repeat(base, 4, axis=0)[:n]
    flip = rng.random((n, m)) < 0.3
    g = np.where(flip, rng.integers(0, 3, size=(n, m)), g).astype(float)
    z = g - g.mean(0)
    k = z @ z.T / max(1.0, float((g.mean(0) / 2 * (1 - g.mean(0) / 2)).sum() * 2))
    v = 0.4 * k + 0.2 * k * k + 0.4 * np.eye(n)
    x = np.column_stack([np.ones(n)] + [rng.integers(0, 2, n) for _ in range(ncov)]).astype(float)
    vi = np.linalg.inv(v)
    vx = vi @ x
    p = vi - vx @ np.linalg.solve(x.T @ vx, vx.T)
    p = 0.5 * (p + p.T)
    trp = np.trace(p)
    return p + 4.0 * trp / n * np.ones((n, n)) / n


@pytest.mark.parametrize("n,ncov,ne", [(600, 0, 200), (2000, 0, 385), (2000, 3, 385), (1237, 2, 64)])
def test_eig_bottom_vs_numpy(n, ncov, ne):
    from gmat_amd import _native as N
    lib = N.ensure_device()
    a = np.ascontiguousarray(_p_matrix(n, 3 * n, ncov, seed=n + ncov))
    w = np.zeros(ne)
    z = np.zeros((ne, n))
    N.check(lib.gmat_probe_eig_bottom(n, N.ptr(a), ne, N.ptr(w), N.ptr(z)), "gmat_probe_eig_bottom")
    wr = np.linalg.eigvalsh(a)[:ne]
    anorm = np.abs(np.linalg.eigvalsh(a)).max()
    np.testing.assert_allclose(w, wr, rtol=0, atol=1e-11 * anorm)
    if ncov:
        assert np.all(np.abs(w[:ncov]) < 1e-10 * anorm)  # the covariates' null directions
    resid = np.abs(z @ a - w[:, None] * z).max()
    assert resid < 1e-9 * anorm, resid
    orth = np.abs(z @ z.T - np.eye(ne)).max()
    assert orth < 1e-8, orth
