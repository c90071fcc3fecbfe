"""The scan plan's partial symmetric eigensolver (gmat_amd/csrc/eig.hip: Chebyshev-filtered subspace
iteration, device Rayleigh-Ritz) against numpy's dense decomposition, on projection matrices P of the kind the plan decomposes (uvlmm_varcom.py:
P = V^-1 - V^-1 X (X'V^-1 X)^-1 X'V^-1, intercept direction lifted as epi_plan.hip eigen_bottom does),
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


def _eig(a, ne, tol, maxit):
    from gmat_amd import _native as N
    import ctypes
    lib = N.ensure_device()
    n = a.shape[0]
    w = np.zeros(ne)
    z = np.zeros((ne, n))
    res = np.zeros(ne)
    it = ctypes.c_int(0)
    N.check(lib.gmat_probe_eig_bottom(n, N.ptr(a), ne, tol, maxit, N.ptr(w), N.ptr(z), N.ptr(res), ctypes.byref(it)),
            "gmat_probe_eig_bottom")
    return w, z, res, it.value


# (n, ncov, ne): the LDS-resident Rayleigh-Ritz (block k <= 192: ne 64, 129) and the global one
@pytest.mark.parametrize("n,ncov,ne", [(600, 0, 200), (2000, 0, 129), (2000, 3, 385), (1237, 2, 64)])
def test_eig_bottom_vs_numpy(n, ncov, ne):
    a = np.ascontiguousarray(_p_matrix(n, 3 * n, ncov, seed=n + ncov))
    w, z, res, iters = _eig(a, ne, 1e-13, 80)
    wall = np.linalg.eigvalsh(a)
    wr = wall[:ne]
    anorm = np.abs(wall).max()
    np.testing.assert_allclose(w, wr, rtol=0, atol=1e-10 * anorm)
    if ncov:
        assert np.all(np.abs(w[:ncov]) < 1e-10 * anorm)  # the covariates' null directions
    resid = np.abs(z @ a - w[:, None] * z).max()
    assert resid < 1e-9 * anorm, resid
    np.testing.assert_allclose(np.linalg.norm(z @ a - w[:, None] * z, axis=1), res, rtol=1e-6, atol=1e-12 * anorm)
    orth = np.abs(z @ z.T - np.eye(ne)).max()
    assert orth < 1e-8, orth
    assert iters < 80


def test_eig_bottom_plan_tolerance():
    """At the plan's tolerance (3e-4 of the Gershgorin bound, <= 16 block iterations) the Ritz values
    bound the true eigenvalues from above and lie within the residual of them (Weyl / Kato)."""
    n, ne = 2000, 129
    a = np.ascontiguousarray(_p_matrix(n, 3 * n, 0, seed=7))
    w, z, res, iters = _eig(a, ne, 3e-4, 16)
    wr = np.linalg.eigvalsh(a)[:ne]
    assert iters <= 16
    assert np.all(w >= wr - 1e-12)
    assert np.all(w - wr <= res.max() + 1e-12)
    orth = np.abs(z @ z.T - np.eye(ne)).max()
    assert orth < 1e-10, orth
