"""Scan-schedule variants of the low-rank screen path give byte-identical results: the compacted
screen (default) against the block-granular one (GMAT_LR_BLOCKS=1: lr_screen_kernel over every
flagged 32-pair block), the pair screen run in chunks beside the later launches (GMAT_PS_CHUNK small,
or 0: all at flush time), and the prefilter's persistent grid against one workgroup per tile
(GMAT_PF_NOLIST) and against a few workgroups looping over many tiles (GMAT_PF_WG).  The default is
checked against the oracle (remma_epiAA.py:71-82 and the epiAD sibling) on sampled rows, every
variant against the default on the whole scan (several launches, so the next-tile prefetch and the
chunked pair screen both run)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VARIANTS = [{"GMAT_LR_BLOCKS": "1"}, {"GMAT_PS_CHUNK": "700"}, {"GMAT_PS_CHUNK": "0"},
            {"GMAT_LR_BLOCKS": "1", "GMAT_PS_CHUNK": "300"},
            {"GMAT_PF_NOLIST": "1"},  # prefilter: one workgroup per tile
            {"GMAT_PF_WG": "8"},      # prefilter: 8 persistent workgroups, ~10 tiles each per launch
            {"GMAT_PF_WG": "24"},
            {"GMAT_LRC_ROWS": "256"},  # compacted scan: 256-row launches (default: 512 at this size)
            {"GMAT_LRC_OPS_CAP": "64"},  # live-pair records overflow: grown and the launches rerun
            {"GMAT_LRC_MIN_LAUNCHES": "1"},  # one launch of all rows (no prefilter-ahead pipeline)
            {"GMAT_SEG_MAX": "1"},  # refine8 / pair_mxr without row-block segments
            {"GMAT_LRC_J4": "1"}]  # compacted screen reading the j side's 4-bit nibble planes


@pytest.fixture(scope="module")
def cohort(tmp_path_factory):
    from gmat_amd import synth
    from oracle import gmat_oracle as O
    d = tmp_path_factory.mktemp("lrv")
    prefix = os.path.join(str(d), "c")
    synth.make_cohort(prefix, 700, 2900, seed=31)  # n_pad 768: six 128-individual stages
    snp = O.read_plink(prefix)
    ka = O.agmat(snp)
    y, x, col, nid = O.design_matrix(prefix + ".pheno", prefix)
    pvp, py = O.projection(y, x, col, nid, [ka, ka * ka], np.array([0.4, 0.2, 0.4]))
    return prefix, snp, pvp, py


def _scan(plan, kind, rows, p_cut, env):
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


@pytest.mark.parametrize("kind", ["AA", "AD"])
def test_schedule_variants_identical(cohort, kind):
    from gmat_amd.plink import Geno
    from gmat_amd.remma._scan import EpiPlan
    from oracle import gmat_oracle as O
    prefix, snp, pvp, py = cohort
    m = snp.shape[1]
    rows = np.arange(m - 1 if kind == "AA" else m, dtype=np.int64)
    p_cut = 1e-4  # automatic level: the low-rank screen
    with Geno(prefix) as g, EpiPlan(g, pvp, py[:, 0]) as plan:
        assert plan.lowrank_rank() > 0
        ref = _scan(plan, kind, rows, p_cut, {})
        assert plan.stats()["n_slice"] == -1  # the low-rank level ran
        assert ref[0].size > 50
        sample = np.array([0, 3, 700, 1450, 2201, 2897])
        exp = O.epi_scan(kind, snp, pvp, py, snp_lst_0=sample, p_cut=p_cut)
        sel = np.isin(ref[0], sample)
        np.testing.assert_array_equal(ref[0][sel], exp[:, 0].astype(np.int64))
        np.testing.assert_array_equal(ref[1][sel], exp[:, 1].astype(np.int64))
        np.testing.assert_allclose(ref[5][sel], exp[:, 4], rtol=1e-8)
        for env in VARIANTS:
            got = _scan(plan, kind, rows, p_cut, env)
            for u, v in zip(got, ref):
                np.testing.assert_array_equal(u, v, err_msg=str(env))
