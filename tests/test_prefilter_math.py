"""CPU checks of the algebra behind the scan's spectral prefilter (epi_*.hip).

The device code never forms e = x_i o x_j: it expands |e|^2 and 1'e into exact integer code
products (a.b, a^2.b, a.b^2, a^2.b^2) and per-SNP sums, and bounds e'Pe from below by a
Cholesky-certified spectral inequality.  These tests restate both in numpy and check them on
random codes and on a relationship-style projection matrix.
"""
import numpy as np


def expanded_norms(a, b, al, be):
    """|e|^2 and 1'e for e = (a - al) o (b - be) from the code products (prefilter epilogue)."""
    n = a.size
    sab, sa2b, sab2, sa2b2 = a @ b, (a * a) @ b, a @ (b * b), (a * a) @ (b * b)
    ca, ca2, cb, cb2 = a.sum(), (a * a).sum(), b.sum(), (b * b).sum()
    ee = (sa2b2 - 2 * be * sa2b + be * be * ca2 - 2 * al * sab2 + 4 * al * be * sab - 2 * al * be * be * ca
          + al * al * cb2 - 2 * al * al * be * cb + n * al * al * be * be)
    se = sab - be * ca - al * cb + n * al * be
    return ee, se


def test_expansion_matches_direct():
    rng = np.random.default_rng(3)
    for _ in range(50):
        n = int(rng.integers(5, 300))
        a = rng.integers(0, 3, n).astype(np.float64)
        b = rng.integers(0, 3, n).astype(np.float64)
        al, be = rng.uniform(0, 2, 2)
        e = (a - al) * (b - be)
        ee, se = expanded_norms(a, b, al, be)
        np.testing.assert_allclose(ee, e @ e, rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(se, e.sum(), rtol=1e-12, atol=1e-9)


def _projection(n, rng):
    """P = V^-1 - V^-1 1 (1'V^-1 1)^-1 1'V^-1 for V = 0.4 K + 0.2 K*K + 0.4 I (P 1 = 0)."""
    g = rng.integers(0, 3, (n, 4 * n)).astype(np.float64)
    g -= g.mean(1, keepdims=True)
    k = g @ g.T / g.shape[1]
    v = 0.4 * k + 0.2 * k * k + 0.4 * np.eye(n)
    vi = np.linalg.inv(v)
    one = np.ones((n, 1))
    return vi - vi @ one @ np.linalg.inv(one.T @ vi @ one) @ one.T @ vi


def certify(p, iters=40):
    """Bisection on mu with the Cholesky of A = P + (mu + tau) 11'/n - mu I (gmat_epi_create)."""
    n = p.shape[0]
    tr = np.trace(p)
    tau0 = 1e-8 * tr / n
    lo, hi = 0.0, 2.0 * tr / n
    for _ in range(iters):
        mid = 0.5 * (lo + hi)
        a = p + (mid + tau0 + 1e-6 * mid) / n - mid * np.eye(n)
        try:
            np.linalg.cholesky(a)
            lo = mid
        except np.linalg.LinAlgError:
            hi = mid
    eps = 2.0 * (n + 1) * 2.0 ** -53 * (tr + tau0 + 1e-6 * lo + lo * (1 - n)) * 1.01
    return lo, tau0 + 1e-6 * lo, eps


def test_certified_bound_holds():
    rng = np.random.default_rng(5)
    n = 120
    p = _projection(n, rng)
    mu, tau, eps = certify(p)
    lam = np.linalg.eigvalsh(p)
    assert abs(lam[0]) < 1e-10                  # the intercept direction
    assert 0.9 * lam[1] < mu <= lam[1] * (1 + 1e-6)  # mu is the smallest eigenvalue on 1-perp
    for _ in range(2000):
        a = rng.integers(0, 3, n).astype(np.float64)
        b = rng.integers(0, 3, n).astype(np.float64)
        al, be = rng.uniform(0, 2, 2)
        e = (a - al) * (b - be)
        ee, se = expanded_norms(a, b, al, be)
        vlo = mu * (ee - se * se / n) - tau * se * se / n - eps * ee
        assert e @ p @ e >= vlo - 1e-9 * abs(vlo)
    # adversarial directions: the eigenvectors themselves (the bound must hold with equality-ish)
    _, q = np.linalg.eigh(p)
    for k in range(1, 6):
        e = q[:, k]
        assert e @ p @ e >= mu * (e @ e - e.sum() ** 2 / n) - tau * e.sum() ** 2 / n - eps * (e @ e) - 1e-12


def _projection_x(n, x, rng):
    """P = V^-1 - V^-1 X (X'V^-1 X)^-1 X'V^-1 (P X = 0: null directions besides 1)."""
    g = rng.integers(0, 3, (n, 4 * n)).astype(np.float64)
    g -= g.mean(1, keepdims=True)
    k = g @ g.T / g.shape[1]
    v = 0.4 * k + 0.2 * k * k + 0.4 * np.eye(n)
    vi = np.linalg.inv(v)
    return vi - vi @ x @ np.linalg.inv(x.T @ vi @ x) @ x.T @ vi


def certify_cov(p, k0_max=4):
    """gmat_epi_create's covariate-design certificate: U = eigenvectors of P + 4 tr(P)/n 11'/n with
    eigenvalue ~ 0; mu from the next eigenvalue with a few candidates, certified by the Cholesky of
    A = P + (mu + tau) 11'/n + (mu + tau) U U' - mu I."""
    n = p.shape[0]
    tr = np.trace(p)
    lam, z = np.linalg.eigh(p + 4 * tr / n * np.ones((n, n)) / n)
    k0 = int(np.sum(lam < 1e-9 * tr / n))
    assert k0 <= k0_max
    u = z[:, :k0].T
    tau0 = 1e-8 * tr / n
    for f in (1 - 2e-3, 1 - 2e-2, 0.9, 0.7):
        mu = f * lam[k0]
        tau = tau0 + 1e-6 * mu
        a = p + (mu + tau) / n + (mu + tau) * u.T @ u - mu * np.eye(n)
        try:
            np.linalg.cholesky(a)
            break
        except np.linalg.LinAlgError:
            mu = 0.0
    eps = 2.0 * (n + 1) * 2.0 ** -53 * abs(tr + (mu + tau) * (1 + k0) - n * mu) * 1.01 + n * (k0 + 4) * 2.0 ** -53 * (
        np.abs(p).max() + mu + 2 * (mu + tau) / n + (mu + tau))
    return mu, tau, mu + tau, eps, u


def test_covariate_certificate_and_int8_images():
    """With covariates the intercept-only certificate gives mu ~ 0; the directions U restore mu
    to the smallest eigenvalue off span(X), and the per-pair bound with one-slice int8 images of
    (a o u_k) (error <= sU csum_b / 2) holds on random and adversarial pairs."""
    rng = np.random.default_rng(11)
    n = 150
    x = np.column_stack([np.ones(n), rng.integers(0, 2, n), rng.uniform(90, 130, n)])
    p = _projection_x(n, x, rng)
    mu0, _, _ = certify(p, iters=30)
    assert mu0 < 1e-6  # intercept-only certificate: nothing to screen with
    mu, tau, ku, eps, u = certify_cov(p)
    assert u.shape[0] == 2
    lam = np.linalg.eigvalsh(p)
    assert mu > 0.9 * lam[3] and mu > 1e3 * eps  # lam[0..2] ~ 0: the three columns of X
    np.testing.assert_allclose(np.abs(u.sum(1)), 0.0, atol=1e-9)  # the directions are orthogonal to 1
    for trial in range(1500):
        a = rng.integers(0, 3, n).astype(np.float64)
        b = rng.integers(0, 3, n).astype(np.float64)
        al, be = rng.uniform(0, 2, 2)
        if trial % 3 == 0:  # adversarial: e close to span(X)
            t = x @ rng.standard_normal(3)
            a = np.clip(np.rint(1 + t / np.abs(t).max()), 0, 2)
            b = np.ones(n) * 2
        e = (a - al) * (b - be)
        ee, se = expanded_norms(a, b, al, be)
        u2 = 0.0
        for k in range(u.shape[0]):
            v = a * u[k]
            su = np.abs(v).max() / 127 if np.abs(v).max() > 0 else 1.0
            q = np.clip(np.rint(v / su), -127, 127)
            ck = su * (q @ b) - be * (a @ u[k]) - al * (u[k] @ b) + al * be * u[k].sum()
            err = 0.5 * su * b.sum() * (1 + 1e-9) + 1e-12 * (abs(su * (q @ b)) + abs(be * (a @ u[k])) + abs(al * (u[k] @ b)))
            assert abs(ck - u[k] @ e) <= err
            u2 += (abs(ck) + err) ** 2
        vlo = (mu - eps) * ee - (mu + tau) * se * se / n - ku * u2
        assert e @ p @ e >= vlo - 1e-9 * abs(vlo)
