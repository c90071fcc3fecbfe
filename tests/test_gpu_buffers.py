"""Plan-buffer reuse and the int8 refine's anchor (round-5 review items).

* Live-block entries of the compacted scan (epi_scan.hip scan_lowrank alloc_sets): when the rows per launch
  grow within one device-memory size class, the cache hands the same block back; its rows past the old
  size must not be read as live blocks.  A plan that scanned at 640 rows per launch leaves tagged
  entries in its block; a second plan then scans at 512 and again at 640 rows per launch -- every scan
  must equal the oracle (remma_epiAA.py:71-82) on sampled rows and the first plan's hits.
* The int8-slice refine (refine8 / refine8w) against the fp64 MFMA refine (GMAT_REFINE64) on the same
  pair lists, for n_pad <= 2,048 (w in registers) and the wide path (n_pad > 2,048): the exhaustive-hit
  golden of the configs[2] bench is refine8 output, so this pins refine8 to the fp64 form directly.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _env_scan(plan, kind, rows, p_cut, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return plan.scan(kind, rows, p_cut)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _cohort(n, m, seed):
    from gmat_amd import synth
    from oracle import gmat_oracle as O
    geno = synth.simulate_genotypes(n, m, seed=seed)
    snp = np.ascontiguousarray(geno.T, dtype=np.float64)
    ka = O.agmat(snp[:, : min(m, 3000)])
    rng = np.random.default_rng(seed)
    y = 1.0 + rng.standard_normal(n)
    col = np.arange(n)
    pvp, py = O.projection(y, np.ones((n, 1)), col, n, [ka, ka * ka], np.array([0.4, 0.2, 0.4]))
    body = np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8)
    return body, snp, pvp, py[:, 0]


def test_live_entries_after_rows_per_launch_grow():
    from gmat_amd.plink import Geno
    from gmat_amd.remma._scan import EpiPlan
    from oracle import gmat_oracle as O
    n, m = 700, 10000  # 32-column blocks: 313 per row; 512 and 640 rows of entries share a 2 MiB class
    body, snp, pvp, py = _cohort(n, m, 41)
    rows = np.arange(m - 1, dtype=np.int64)
    p_cut = 1e-4
    with Geno(body=body, n_id=n, n_snp=m) as g:
        with EpiPlan(g, pvp, py) as p1:
            ref = _env_scan(p1, "AA", rows, p_cut, {"GMAT_LRC_ROWS": "640"})
            assert p1.stats()["n_slice"] == -1 and p1.stats()["launches"] >= 8
        with EpiPlan(g, pvp, py) as p2:
            small = _env_scan(p2, "AA", rows, p_cut, {"GMAT_LRC_ROWS": "512"})
            grown = _env_scan(p2, "AA", rows, p_cut, {"GMAT_LRC_ROWS": "640"})
    assert ref[0].size > 20
    sample = np.array([0, 5, 511, 512, 639, 640, 4999, 9997])
    exp = O.epi_scan("AA", snp, pvp, py.reshape(-1, 1), snp_lst_0=sample, p_cut=p_cut)
    sel = np.isin(ref[0], sample)
    np.testing.assert_array_equal(np.column_stack([ref[0][sel], ref[1][sel]]), exp[:, :2].astype(np.int64))
    for got in (small, grown):
        for u, v in zip(got, ref):
            np.testing.assert_array_equal(u, v)


@pytest.mark.parametrize("n", [700, 2200])  # n_pad 768: refine8_kernel; 2,304: refine8w_kernel
def test_refine8_matches_fp64_refine(n):
    from gmat_amd.plink import Geno
    from gmat_amd.remma._scan import EpiPlan
    from oracle import gmat_oracle as O
    m = 600
    body, snp, pvp, py = _cohort(n, m, 43 + n)
    rng = np.random.default_rng(n)
    pairs = np.column_stack([rng.integers(0, m, 3000), rng.integers(0, m, 3000)]).astype(np.int64)
    pairs[:5] = [[0, 1], [3, 3], [m - 1, 0], [m - 2, m - 1], [7, 7]]
    with Geno(body=body, n_id=n, n_snp=m) as g, EpiPlan(g, pvp, py) as plan:
        for kind in ("AA", "AD", "DD"):
            e8, v8, c8, p8 = plan.pairs(kind, pairs)
            os.environ["GMAT_REFINE64"] = "1"
            try:
                e64, v64, c64, p64 = plan.pairs(kind, pairs)
            finally:
                os.environ.pop("GMAT_REFINE64", None)
            ok = np.isfinite(v64) & (v64 != 0)
            assert ok.sum() > 2500
            np.testing.assert_array_equal(np.isfinite(v8), np.isfinite(v64))
            # eff: the same fp64 dot product summed in another order (1e-12 of the largest |eff|)
            np.testing.assert_allclose(e8, e64, rtol=1e-10, atol=1e-12 * np.abs(e64).max())
            # var: ~1e-15 relative, except where it cancels to a small value (then 1e-13 of the largest)
            np.testing.assert_allclose(v8[ok], v64[ok], rtol=1e-13, atol=1e-13 * np.abs(v64).max())
            # p: the cancelling pairs' var moves p by up to ~1e-9 (a small var's relative error)
            np.testing.assert_allclose(p8[ok], p64[ok], rtol=1e-8, atol=1e-9)
        # and both against the oracle on a subset
        o_eff, o_var, o_chi, o_p = O.epi_pair("AA", snp, pvp, py.reshape(-1, 1), pairs[:200])
        e8, v8, c8, p8 = plan.pairs("AA", pairs[:200])
        fin = np.isfinite(o_chi)
        np.testing.assert_allclose(v8[fin], o_var[fin], rtol=1e-10, atol=1e-12 * np.abs(o_var).max())
        np.testing.assert_allclose(e8[fin], o_eff[fin], rtol=1e-9, atol=1e-12 * np.abs(o_eff).max())
