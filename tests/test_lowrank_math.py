"""CPU checks of the low-rank spectral screen (epi_plan.hip lr_setup / lr_screen_kernel).

The device screen bounds var = e'Pe from below by
    lam (|e|^2 - (1'e)^2/n) - tau (1'e)^2/n - eps |e|^2 - sum_r d_r (B_r'e)^2,
B the bottom eigenvectors of P, D = diag(d), with Q = fp6(B sqrt(D)) (what the MFMA multiplies)
and lam certified by a Cholesky of P - lam I + (lam + tau) 11'/n + Q Q'.  It never forms e:
Q_r'e is expanded as Q_r'(a o b) - beta (Q_r'a - alpha Q_r'1) - alpha Q_r'b.  These tests restate the fp6
quantiser, the certificate and the expansion in numpy and check the bound on code vectors.
"""
import numpy as np

from test_prefilter_math import _projection


def fp6_block(v):
    """fp6 e2m3 values with one e8m0 scale per 32 entries (fp6_block in epi_plan.hip)."""
    mx = np.abs(v).max()
    if mx == 0:
        return np.zeros_like(v)
    e = int(np.ceil(np.log2(mx / 7.5)))
    while np.ldexp(7.5, e) < mx:
        e += 1
    while np.ldexp(7.5, e - 1) >= mx:
        e -= 1
    y = np.ldexp(v, -e)
    ay = np.abs(y)
    q = np.where(ay < 2, np.rint(ay * 8) / 8, np.where(ay < 4, np.rint(ay * 4) / 4, np.rint(ay * 2) / 2))
    return np.ldexp(np.sign(y) * q, e)


def quantise(u):
    """columns of u (n x R) quantised in 32-row blocks, as the B' tile images hold them."""
    out = np.zeros_like(u)
    for r in range(u.shape[1]):
        for k0 in range(0, u.shape[0], 32):
            out[k0:k0 + 32, r] = fp6_block(u[k0:k0 + 32, r])
    return out


def certify_lowrank(p, rank, kappa=0.7, iters=30):
    """lr_setup: Q(lam) = fp6(u_r sqrt(d_r(lam))) and a bisected Cholesky of
    P - lam I + (lam + tau) 11'/n + Q Q'.  Returns lam, tau and the certified Q."""
    n = p.shape[0]
    w, v = np.linalg.eigh(p + 4.0 * np.trace(p) / n * np.ones((n, n)) / n)
    lam_r, top = w[:rank], w[rank]
    tau = 0.5 * top

    def q_of(lam):
        return quantise(v[:, :rank] * np.sqrt(np.maximum(lam - lam_r, 0) * (1 + kappa)))

    lo, hi = 0.0, 1.3 * top
    for _ in range(iters):
        mid = 0.5 * (lo + hi)
        q = q_of(mid)
        a = p - mid * np.eye(n) + (mid + tau) / n + q @ q.T
        try:
            np.linalg.cholesky(a)
            lo = mid
        except np.linalg.LinAlgError:
            hi = mid
    return lo, tau, q_of(lo)


def test_fp6_grid():
    v = np.array([7.5, -7.4, 3.3, 0.06, 0.0, -1.9375] + [0.0] * 26)
    q = fp6_block(v)
    # steps 1/8 below 2 (half-even), 1/4 below 4, 1/2 up to 7.5
    assert q[0] == 7.5 and q[1] == -7.5 and q[2] == 3.25 and q[3] == 0.0 and q[4] == 0.0 and q[5] == -2.0


def test_lowrank_bound_holds_and_beats_the_prefilter():
    rng = np.random.default_rng(11)
    n, rank = 160, 64
    p = _projection(n, rng)
    lam, tau, b = certify_lowrank(p, rank)
    w = np.linalg.eigvalsh(p)
    mu0 = w[1]  # the prefilter's ceiling: smallest eigenvalue on 1-perp
    assert lam > 1.2 * mu0 and lam > 0.95 * w[rank + 1]  # close to the first eigenvalue left out
    one = np.ones(n)
    q1 = b.T @ one
    worst = np.inf
    for _ in range(400):
        a = rng.integers(0, 3, n).astype(np.float64)
        bb = rng.integers(0, 3, n).astype(np.float64)
        al, be = a.mean(), bb.mean()
        e = (a - al) * (bb - be)
        # the kernel's expansion of Q'e: G' = Q'a - alpha Q'1 (left), H = Q'b (right)
        c = b.T @ (a * bb) - be * (b.T @ a - al * q1) - al * (b.T @ bb)
        np.testing.assert_allclose(c, b.T @ e, rtol=1e-9, atol=1e-9)
        ee, se = e @ e, e.sum()
        lb = lam * (ee - se * se / n) - tau * se * se / n - c @ c
        var = e @ p @ e
        assert lb <= var * (1 + 1e-9) + 1e-9
        worst = min(worst, var / max(lb, 1e-300))
    assert worst >= 1.0
