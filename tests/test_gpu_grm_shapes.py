"""GRM int8 SYRK over ragged shapes: the stream-K work list's edges (one stage, a stage past the last
SNP, segments crossing tiles, one tile, a partial last tile, individuals not a multiple of 4), additive
and dominance kinds, against the formula of gmatrix.py:52-66 / :115-130 in fp64 numpy (Z Z' / scale
with the diagonal times 1 + small_val).  The kernel's integer products are exact; the fp64 centring
runs in another order, so the bar is 1e-11 relative to the largest entry."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHAPES = [(3, 1), (5, 127), (64, 128), (255, 129), (257, 385), (700, 9000), (513, 20000)]


def _panel(rng, n, m):
    g = rng.choice(np.array([0, 1, 2], dtype=np.int64), size=(m, n), p=[0.5, 0.3, 0.2])
    g[:, 0], g[:, -1] = 0, 2  # every SNP polymorphic (scale > 0)
    code = np.array([0, 2, 3], dtype=np.uint8)[g]  # PLINK: 00 hom, 10 het, 11 other hom
    nb = (n + 3) // 4
    pad = np.zeros((m, 4 * nb), dtype=np.uint8)
    pad[:, :n] = code
    c = pad.reshape(m, nb, 4)
    body = (c[:, :, 0] | (c[:, :, 1] << 2) | (c[:, :, 2] << 4) | (c[:, :, 3] << 6)).astype(np.uint8).ravel()
    return g, body


def _expected(g, kind, small_val):
    n = g.shape[1]
    p = g.sum(axis=1) / (2.0 * n)
    s = 2.0 * p * (1.0 - p)
    if kind == 0:
        z = g - (2.0 * p)[:, None]
        scale = s.sum()
    else:
        z = (g == 1).astype(np.float64) - s[:, None]
        scale = (s * (1.0 - s)).sum()
    k = z.T @ z / scale
    k[np.diag_indices(n)] *= 1.0 + small_val
    return k, scale


@pytest.mark.parametrize("n,m", SHAPES)
def test_grm_shapes(n, m):
    from gmat_amd import _native as N
    from gmat_amd.plink import Geno
    lib = N.ensure_device()
    rng = np.random.default_rng(n * 7919 + m)
    g, body = _panel(rng, n, m)
    geno = Geno(body=body, n_id=n, n_snp=m)
    try:
        for kind in (0, 1):
            k = np.empty((n, n))
            sc = ctypes.c_double()
            N.check(lib.gmat_grm(geno.handle, kind, 0.001, N.ptr(k), ctypes.byref(sc)), "gmat_grm")
            exp, scale = _expected(g, kind, 0.001)
            assert sc.value == pytest.approx(scale, rel=1e-12)
            # a diagonal tile's two triangles are centred by different lanes ((g - r_a) - r_b against
            # (g - r_b) - r_a): symmetric to rounding, as the reference's fp64 product
            np.testing.assert_allclose(k, k.T, rtol=0, atol=1e-14 * max(1.0, np.abs(k).max()))
            np.testing.assert_allclose(k, exp, rtol=0, atol=1e-11 * max(1.0, np.abs(exp).max()))
    finally:
        geno.close()
