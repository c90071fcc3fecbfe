"""Oracle anchor of the full-size hit set.

tests/golden/cfg3_exhaustive_hits_AA_2000x50000.npz -- the hits bench.py checks every timed step
against -- was written by the HIP exhaustive level (every pair refined, no screen).  Here the
oracle's own chain, on the box's host CPU, re-derives those numbers for the bench cohort
(configs[2]: 2,000 x 50,000, seed 1, p_cut 1e-5) without any device result in between:

* GRM: O.agmat of the decoded genotypes (gmatrix.py:52-66);
* P, Py: O.projection with the bench's model [A, AxA] and the simulated phenotype
  (remma_epiAA.py:33-49);
* pair statistics: O.epi_pair (remma_epiAA.py:71-82 formula) over all 10,932 recorded hits, every
  pair the device scan finds with p < 2e-5 (the ~11k pairs just above the threshold) and 50,000
  random pairs of the triangle.

The oracle's hit set over those pairs must equal the recorded one (a pair whose p lies within
1e-9 relative of p_cut may fall either side: the GRM sums in another order), and eff / var / chi /
p of the recorded hits must agree to 1e-8 relative."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden", "cfg3_exhaustive_hits_AA_2000x50000.npz")
P_CUT = 1e-5


def test_full_size_hits_against_the_oracle():
    sys.path.insert(0, REPO)
    import bench
    from oracle import gmat_oracle as O  # the checker
    from gmat_amd.remma._scan import EpiPlan
    from tools.full_triangle import cohort_fingerprint
    n, m = 2000, 50000
    var = np.array([0.4, 0.2, 0.4])
    geno, g, pvp, py, ka, y = bench.build_inputs(n, m, 1, var, 0, 1)
    d = np.load(GOLD)
    assert bytes(d["fingerprint"]).hex() == cohort_fingerprint(g, pvp, py), "not the bench cohort"
    gold = {(int(a), int(b)): k for k, (a, b) in enumerate(zip(d["i"], d["j"]))}
    assert len(gold) == 10932

    # the device scan at twice the threshold: the pairs just above p_cut (screened + exact refine;
    # the screens are audited against the exhaustive level over the whole triangle elsewhere)
    with EpiPlan(g, pvp, py) as plan:
        near = plan.scan("AA", np.arange(m - 1), 2 * P_CUT)
    near_pairs = set(zip(near[0].tolist(), near[1].tolist()))
    assert set(gold) <= near_pairs
    rng = np.random.default_rng(2024)
    i = rng.integers(0, m - 1, 200000)
    j = rng.integers(0, m, 200000)
    keep = i < j
    rand_pairs = set()
    for pr in zip(i[keep].tolist(), j[keep].tolist()):
        rand_pairs.add(pr)
        if len(rand_pairs) == 50000:
            break
    pairs = np.array(sorted(set(gold) | near_pairs | rand_pairs), dtype=np.int64)
    g.close()

    # the oracle's chain from the genotypes: GRM, P / Py, pair statistics (fp64 numpy / host BLAS)
    snp = np.ascontiguousarray(geno.T, dtype=np.float64)
    del geno
    ka_o = O.agmat(snp)
    np.testing.assert_allclose(ka_o, ka, rtol=1e-10, atol=1e-12)  # the device GRM the bench used
    pvp_o, py_o = O.projection(y, np.ones((n, 1)), np.arange(n), n, [ka_o, ka_o * ka_o], var)
    py_o = py_o[:, 0]
    np.testing.assert_allclose(pvp_o, pvp, rtol=1e-7, atol=1e-12 * np.abs(pvp).max())
    a, _ = O.codings(snp)
    del snp
    res = np.zeros((pairs.shape[0], 4))
    for t in range(0, pairs.shape[0], 4096):
        pr = pairs[t:t + 4096]
        e = a[:, pr[:, 0]] * a[:, pr[:, 1]]
        eff = e.T @ py_o
        var_ = np.sum(e * (pvp_o @ e), axis=0)
        chi = eff * eff / var_
        res[t:t + 4096] = np.column_stack([eff, var_, chi, np.zeros_like(chi)])
    from scipy.stats import chi2
    res[:, 3] = chi2.sf(res[:, 2], 1)

    hit = res[:, 3] < P_CUT
    border = np.abs(res[:, 3] - P_CUT) <= 1e-9 * P_CUT
    oracle_hits = {tuple(p) for p in pairs[hit & ~border].tolist()}
    gold_core = {k for k in gold if not border[np.searchsorted(pairs[:, 0] * m + pairs[:, 1], k[0] * m + k[1])]}
    assert oracle_hits == gold_core, (len(oracle_hits - gold_core), len(gold_core - oracle_hits))
    idx = np.searchsorted(pairs[:, 0] * m + pairs[:, 1], d["i"].astype(np.int64) * m + d["j"].astype(np.int64))
    np.testing.assert_array_equal(pairs[idx, 0], d["i"])
    for col, name in enumerate(("eff", "var", "chi", "p")):
        np.testing.assert_allclose(d[name], res[idx, col], rtol=1e-8, err_msg=name)
    n_near = len(near_pairs) - len(gold)
    assert n_near > 5000 and len(rand_pairs) == 50000
    print("oracle anchor: %d recorded hits, %d pairs in [p_cut, 2 p_cut), %d random pairs, %d on the border"
          % (len(gold), n_near, len(rand_pairs), int(border.sum())))
