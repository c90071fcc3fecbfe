"""The int8-slice refine (refine8_kernel + refine8_side_kernel in csrc/epi_*.hip) restated in numpy:
the block-upper slice images, the exact integer quadratic forms per slice, the expansion of e'Pe
around the integer codes, and the tile count r8_toff.  The statistic it feeds is the reference's
var = e'Pe of remma_epiAA.py:71-82; this checks that the restated arithmetic reproduces it to the
bound the kernel's comment states (|w'Rw| <= 8e-16 qmax |w|_1^2 after 7 slices)."""
import numpy as np

R8_S = 7


def r8_toff(kb, ns):
    h = kb >> 1
    return kb * ns - (h * h if kb & 1 else h * (h - 1))


def block_upper_slices(P, unit):
    """The slices of P' = P_off with blocks right of the diagonal (32-row granularity) doubled and
    those left of it zero, cut at `unit` (r8_image_kernel)."""
    n = P.shape[0]
    blk = np.arange(n) // 32
    f = np.where(blk[None, :] > blk[:, None], 2.0, np.where(blk[None, :] == blk[:, None], 1.0, 0.0))
    r = np.where(np.eye(n, dtype=bool), 0.0, P) * f / unit
    out = []
    for _ in range(R8_S):
        q = np.rint(r)
        assert np.all(np.abs(q) <= 127)
        out.append(q.astype(np.int64))
        r = (r - q) * 128.0
    return out


def test_tile_offsets():
    for n_pad in (128, 256, 640, 2048):
        NS, NB = n_pad // 64, n_pad // 32
        k = 0
        for kb in range(NB + 1):
            assert r8_toff(kb, NS) == k
            if kb < NB:
                k += NS - kb // 2


def test_sliced_quadratic_form_is_the_fp64_one():
    rng = np.random.default_rng(3)
    n = 256
    a = rng.standard_normal((n, n))
    P = (a @ a.T) / n + np.eye(n)
    P /= np.abs(P).max()
    qmax = np.abs(P - np.diag(np.diag(P))).max()
    unit = 2.0 * qmax / 127.0
    A = block_upper_slices(P, unit)
    for _ in range(20):
        wa = rng.integers(0, 3, n)
        wb = rng.integers(0, 3, n)
        w = wa * wb
        # per slice an exact integer (the MFMA's int32 sums, folded in int32 per row tile)
        T = [int(w @ (As @ w)) for As in A]
        assert all(abs(t) < 2 ** 53 for t in T)
        tot = 0.0
        for t in reversed(T):
            tot = tot / 128.0 + float(t)
        got = unit * tot
        exact = float(w @ ((P - np.diag(np.diag(P))) @ w))
        bound = 8e-16 * qmax * float(np.abs(w).sum()) ** 2 + 1e-15 * abs(exact)
        assert abs(got - exact) <= bound, (got, exact, bound)


def test_expansion_around_integer_codes():
    """e'Pe = w'P_off w + sum_q P_qq w_q^2 + 2 v'Pw + v'Pv with e = (a - alpha)(b - beta), w = a o b,
    v = -beta a - alpha b + alpha beta 1 (the pair screen's and refine8_side_kernel's terms)."""
    rng = np.random.default_rng(5)
    n = 200
    a_ = rng.standard_normal((n, n))
    P = a_ @ a_.T / n
    for _ in range(10):
        a = rng.integers(0, 3, n).astype(float)
        b = rng.integers(0, 3, n).astype(float)
        al, be = a.mean(), b.mean()
        e = (a - al) * (b - be)
        w = a * b
        z = P @ np.ones(n)
        ua, ub = P @ a, P @ b
        poff = P - np.diag(np.diag(P))
        s1 = w @ (al * be * z - be * ua - al * ub)
        var = (w @ poff @ w + np.diag(P) @ (w * w) + 2 * s1 + be * be * (a @ ua) + al * al * (b @ ub) +
               (al * be) ** 2 * (np.ones(n) @ z) + 2 * al * be * (a @ ub) - 2 * al * be * be * (a @ z) -
               2 * al * al * be * (b @ z))
        np.testing.assert_allclose(var, e @ P @ e, rtol=1e-12)
