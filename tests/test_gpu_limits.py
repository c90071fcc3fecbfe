"""Scans past the single-plan limits (epi_seg.hip, epi_plan.hip): the reference's loop
(remma_epiAA.py:35-82, remma_epiAD.py:66-87, remma_epiDD.py:68-86) has no size limit, so neither may
the drop-in.

* More than 8,192 individuals (n = 8,500, n_pad 8,704): the plan has no screens (the int8 slice
  screen's 24-bit sums and the pair screen's LDS planes stop at 8,192) and refines every pair exactly.
  Every AA / AD / DD pair (1.1-2.25 M per kind) is checked against the independent fp64 MFMA refine
  (the reference formula e'Pe with P in fp64), and sampled rows against the CPU oracle.
* SNP segments: GMAT_SEG_SNPS forces a plan cut into segments at sizes one plan could hold; its hits,
  pair statistics and audit bounds are byte-identical to the unsegmented plan's, on the configs[2]
  cohort's stratified rows and on whole scans of a smaller cohort.
* The real limit: 2,000 individuals x 1.1 M SNPs (2 m n_pad = 4.5e9 bytes > 2^32, three segments) --
  the SNPs are a 50,000-SNP cohort repeated 22 times, so every pair's statistics are a pair of the base
  cohort (or a SNP with itself) and the oracle on the base cohort predicts every hit.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _setenv(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    return old


def _restore(old):
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _projection(snp, seed, n_grm=3000):
    from oracle import gmat_oracle as O
    n = snp.shape[0]
    ka = O.agmat(snp[:, :n_grm])
    rng = np.random.default_rng(seed)
    y = 1.0 + rng.standard_normal(n)
    pvp, py = O.projection(y, np.ones((n, 1)), np.arange(n), n, [ka, ka * ka], np.array([0.4, 0.2, 0.4]))
    return pvp, py[:, 0]


def test_more_than_8192_individuals_every_pair():
    """n = 8,500: the exhaustive int8-slice refine (refine8w_kernel) against the independent fp64 MFMA
    refine (GMAT_REFINE64: e'Pe with P in fp64, the reference formula) on EVERY AA / AD / DD pair
    (identical hit sets at p_cut 1e-3, var within 1e-12), and the hits of sampled rows against the
    CPU oracle."""
    from gmat_amd import synth
    from gmat_amd.plink import Geno
    from gmat_amd.remma._scan import EpiPlan
    from oracle import gmat_oracle as O
    n, m, p_cut = 8500, 1500, 1e-3
    geno = synth.simulate_genotypes(n, m, seed=61)
    snp = np.ascontiguousarray(geno.T, dtype=np.float64)
    pvp, py = _projection(snp, 61, n_grm=m)
    body = np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8)
    with Geno(body=body, n_id=n, n_snp=m) as g, EpiPlan(g, pvp, py) as plan:
        lay = plan.layout()
        assert lay["exhaustive_only"] and lay["segments"] == 1, lay
        for kind in ("AA", "AD", "DD"):
            rows = np.arange(m if kind == "AD" else m - 1, dtype=np.int64)
            hi, hj, eff, var, chi, p = plan.scan(kind, rows, p_cut)
            st = plan.stats()
            assert st["pairs"] == (m * m if kind == "AD" else m * (m - 1) // 2), st
            assert hi.size > 20, (kind, hi.size)
            # every pair, both refines
            ii, jj = np.meshgrid(rows, np.arange(m), indexing="ij")
            allp = np.column_stack([ii.ravel(), jj.ravel()])
            if kind != "AD":
                allp = allp[allp[:, 1] > allp[:, 0]]
            e8, v8, c8, p8 = plan.pairs(kind, allp)
            old = _setenv({"GMAT_REFINE64": "1"})
            try:
                e64, v64, c64, p64 = plan.pairs(kind, allp)
                h64 = plan.scan(kind, rows, p_cut)
            finally:
                _restore(old)
            np.testing.assert_allclose(e8, e64, rtol=1e-10, atol=1e-12 * np.abs(e64).max())
            np.testing.assert_allclose(v8, v64, rtol=1e-12, atol=1e-13 * np.abs(v64).max())
            near = np.abs(p64 / p_cut - 1) < 1e-9  # decisions within 1e-9 of the threshold may differ
            got = set(zip(hi.tolist(), hj.tolist()))
            exp = set(zip(h64[0].tolist(), h64[1].tolist()))
            amb = set(map(tuple, allp[near].tolist()))
            assert not ((got ^ exp) - amb), (kind, len(got ^ exp))
            # sampled rows against the CPU oracle
            sample = np.array([0, 1, 700, m - 2], dtype=np.int64)
            exo = O.epi_scan(kind, snp, pvp, py.reshape(-1, 1), snp_lst_0=sample, p_cut=p_cut)
            sel = np.isin(hi, sample)
            np.testing.assert_array_equal(np.column_stack([hi[sel], hj[sel]]), exo[:, :2].astype(np.int64))
            np.testing.assert_allclose(np.column_stack([eff[sel], chi[sel], p[sel]]), exo[:, 2:], rtol=1e-8,
                                       atol=1e-300)


def _compare_plans(g, pvp, py, rows_by_kind, p_cuts, pairs, seg_snps):
    from gmat_amd.remma._scan import EpiPlan
    ref, got = {}, {}
    with EpiPlan(g, pvp, py) as plan:
        assert plan.layout()["segments"] == 1
        for kind, rows in rows_by_kind.items():
            for p_cut in p_cuts:
                ref[kind, p_cut] = plan.scan(kind, rows, p_cut)
            ref[kind, "pairs"] = plan.pairs(kind, pairs)
        ref["audit"] = plan.audit("AA", pairs[:500])
    old = _setenv({"GMAT_SEG_SNPS": str(seg_snps)})
    try:
        with EpiPlan(g, pvp, py) as plan:
            lay = plan.layout()
            assert lay["segments"] >= 3 and lay["segment_snps"] <= seg_snps, lay
            for kind, rows in rows_by_kind.items():
                for p_cut in p_cuts:
                    got[kind, p_cut] = plan.scan(kind, rows, p_cut)
                got[kind, "pairs"] = plan.pairs(kind, pairs)
            got["audit"] = plan.audit("AA", pairs[:500])
    finally:
        _restore(old)
    for key in ref:
        if key == "audit":  # bounds from the imported spectral state (equal up to the eigensolver's bits)
            np.testing.assert_allclose(got[key], ref[key], rtol=1e-12)
            continue
        for u, v in zip(ref[key], got[key]):
            np.testing.assert_array_equal(np.asarray(u).view(np.uint64), np.asarray(v).view(np.uint64),
                                          err_msg=str(key))
    return ref


def test_segments_identical_small_cohort():
    """A 2,000 x 12,000 cohort in segments of 4,096 SNPs (3 segments): whole AA scans at the low-rank
    level (p_cut 1e-4) and at the int8 level (1e-2), AD / DD on row subsets, pair statistics across
    segments and the audit bounds are byte-identical to the one-plan results."""
    from gmat_amd import synth
    from gmat_amd.plink import Geno
    n, m = 2000, 12000
    geno = synth.simulate_genotypes(n, m, seed=71)
    snp = np.ascontiguousarray(geno.T, dtype=np.float64)
    pvp, py = _projection(snp, 71)
    body = np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8)
    rng = np.random.default_rng(5)
    pairs = np.column_stack([rng.integers(0, m, 4000), rng.integers(0, m, 4000)]).astype(np.int64)
    sub = np.unique(np.concatenate([np.linspace(0, m - 2, 40).astype(np.int64), [4095, 4096, 8191, 8192]]))
    with Geno(body=body, n_id=n, n_snp=m) as g:
        ref = _compare_plans(g, pvp, py, {"AA": np.arange(m - 1, dtype=np.int64), "AD": sub, "DD": sub},
                             (1e-4, 1e-2), pairs, 4096)
    assert ref["AA", 1e-4][0].size > 100 and ref["AD", 1e-2][0].size > 100


def test_segments_identical_cfg3_rows():
    """configs[2]'s cohort (2,000 x 50,000) in segments of 4,096 SNPs (13 segments): the stratified
    rows of tests/test_gpu_scale.py give byte-identical hits for AA at p_cut 1e-5 and 1e-3, and DD /
    AD at 1e-3."""
    from gmat_amd import synth
    from gmat_amd.plink import Geno
    from gmat_amd.uvlmm.uvlmm_varcom import projection
    from scipy.sparse import identity
    import ctypes
    from gmat_amd import _native as N
    n, m = 2000, 50000
    geno = synth.simulate_genotypes(n, m, seed=1)
    body = np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8)
    lib = N.ensure_device()
    with Geno(body=body, n_id=n, n_snp=m) as g:
        ka = np.empty((n, n))
        sc = ctypes.c_double()
        N.check(lib.gmat_grm(g.handle, 0, 0.001, N.ptr(ka), ctypes.byref(sc)), "gmat_grm")
        rng = np.random.Generator(np.random.PCG64(2))
        y = np.ones(n)
        for k, s in ((ka, 0.4), (ka * ka, 0.2)):
            y += np.sqrt(s) * (np.linalg.cholesky(k + 1e-4 * np.eye(n)) @ rng.standard_normal(n))
        y += np.sqrt(0.4) * rng.standard_normal(n)
        pvp, py = projection(y, np.ones((n, 1)), identity(n, format="csr"), [ka, ka * ka], [0.4, 0.2, 0.4])
        rows = np.unique(np.concatenate([np.linspace(0, m - 2, 22).astype(np.int64), [1, 24999]]))
        pairs = np.column_stack([rows, rows[::-1]]).astype(np.int64)
        ref = _compare_plans(g, pvp, py, {"AA": rows, "DD": rows[::4], "AD": rows[::4]}, (1e-5, 1e-3), pairs, 4096)
    assert ref["AA", 1e-3][0].size > 200


def test_one_plan_below_the_limit():
    """2,000 individuals x 600,000 SNPs (2 m n_pad = 2.46e9 < 2^32): one plan holds the panel (no
    segments), and a row in its last tenth has the oracle's hits on the repeated base cohort."""
    from gmat_amd import synth
    from gmat_amd.plink import Geno
    from gmat_amd.remma._scan import EpiPlan
    from oracle import gmat_oracle as O
    n, m0, reps, p_cut = 2000, 50000, 12, 1e-4
    base = synth.simulate_genotypes(n, m0, seed=81)
    snp0 = np.ascontiguousarray(base.T, dtype=np.float64)
    pvp, py = _projection(snp0, 81)
    body0 = np.frombuffer(synth.pack_bed(base)[3:], dtype=np.uint8).reshape(m0, (n + 3) // 4)
    body = np.tile(body0, (reps, 1)).ravel()
    m = m0 * reps
    i = 11 * m0 + 777
    with Geno(body=body, n_id=n, n_snp=m) as g, EpiPlan(g, pvp, py) as plan:
        lay = plan.layout()
        assert lay["segments"] == 1 and not lay["exhaustive_only"], lay
        hi, hj, eff, var, chi, p = plan.scan("AA", np.array([i], dtype=np.int64), p_cut)
    st = O.epi_pair("AA", snp0, pvp, py.reshape(-1, 1), np.column_stack([np.full(m0, i % m0), np.arange(m0)]))
    j = np.arange(i + 1, m, dtype=np.int64)
    j = j[st[3][j % m0] < p_cut]
    assert j.size > 5
    np.testing.assert_array_equal(hj, j)
    np.testing.assert_allclose(np.column_stack([eff, chi, p]),
                               np.column_stack([st[0][j % m0], st[2][j % m0], st[3][j % m0]]), rtol=1e-8, atol=1e-300)


def test_real_snp_limit_tiled_cohort():
    """2,000 individuals x 1.1 M SNPs: past 2 m n_pad < 2^32, so the plan is cut into segments (three).
    Rows in every segment, AA and AD, checked against the oracle on the 50,000-SNP base cohort the
    panel repeats (pair (i, j) of the panel is pair (i mod 50,000, j mod 50,000) of the base)."""
    from gmat_amd import synth
    from gmat_amd.plink import Geno
    from gmat_amd.remma._scan import EpiPlan
    from oracle import gmat_oracle as O
    n, m0, reps, p_cut = 2000, 50000, 22, 1e-4
    base = synth.simulate_genotypes(n, m0, seed=81)
    snp0 = np.ascontiguousarray(base.T, dtype=np.float64)
    pvp, py = _projection(snp0, 81)
    nb = (n + 3) // 4
    body0 = np.frombuffer(synth.pack_bed(base)[3:], dtype=np.uint8).reshape(m0, nb)
    body = np.tile(body0, (reps, 1)).ravel()
    m = m0 * reps
    rows = np.array([0, 777, m0 - 2, 9 * m0 + 5, 15 * m0 + 31000, m - 3], dtype=np.int64)
    with Geno(body=body, n_id=n, n_snp=m) as g, EpiPlan(g, pvp, py) as plan:
        lay = plan.layout()
        assert lay["segments"] == 3 and not lay["exhaustive_only"], lay
        assert 2 * lay["segment_snps"] * 2 * 2048 < 2 ** 32
        for kind in ("AA", "AD"):
            rr = rows if kind == "AA" else rows[[1, 3]]
            hi, hj, eff, var, chi, p = plan.scan(kind, rr, p_cut)
            exp_i, exp_j, exp_v = [], [], []
            for i in rr:
                i0 = int(i) % m0
                st = O.epi_pair(kind, snp0, pvp, py.reshape(-1, 1), np.column_stack([np.full(m0, i0), np.arange(m0)]))
                j = np.arange(m, dtype=np.int64)
                if kind == "AA":
                    j = j[j > i]
                sel = st[3][j % m0] < p_cut
                exp_i.append(np.full(sel.sum(), i))
                exp_j.append(j[sel])
                exp_v.append(np.column_stack([st[0][j[sel] % m0], st[2][j[sel] % m0], st[3][j[sel] % m0]]))
            ei, ej, ev = np.concatenate(exp_i), np.concatenate(exp_j), np.concatenate(exp_v)
            assert ei.size > 50, (kind, ei.size)
            np.testing.assert_array_equal(np.column_stack([hi, hj]), np.column_stack([ei, ej]))
            np.testing.assert_allclose(np.column_stack([eff, chi, p]), ev, rtol=1e-8, atol=1e-300)
