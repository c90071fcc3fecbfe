"""The reference README's exact-test workflow run UNCHANGED through ``import gmat``
(README.md:94-120: agmat -> np.loadtxt('.agrm0') -> wemai_multi_gmat -> remma_epiAA ->
annotation_snp_pos), on a cohort with missing calls (imputation, process_plink.py:12-25),
two covariates besides the intercept, and an LD file (annotation.py:57-73), against the
outputs the reference itself wrote for the same script and seeds (tests/golden/readme,
make_golden.py readme)."""
import os
import shutil

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

README = os.path.join(os.path.dirname(__file__), "golden", "readme")


def _rows(path):
    lines = open(path).read().splitlines()
    return lines[0], [l.split() for l in lines[1:] if l.strip()]


def _cmp_table(got, exp, n_int, float_cols):
    hg, rg = _rows(got)
    he, re_ = _rows(exp)
    assert hg.split() == he.split()
    assert len(rg) == len(re_), (len(rg), len(re_))
    for a, b in zip(rg, re_):
        assert len(a) == len(b)
        for k, (u, v) in enumerate(zip(a, b)):
            if k in float_cols:
                assert abs(float(u) - float(v)) <= 1e-5 * abs(float(v)) + 1e-300, (k, u, v)
            else:
                assert u == v, (k, u, v)


def test_readme_workflow_through_gmat(tmp_path):
    for name in ("plink.bed", "plink.bim", "plink.fam", "pheno", "plink.ld"):
        shutil.copy(os.path.join(README, name), str(tmp_path))
    cwd = os.getcwd()
    os.chdir(str(tmp_path))
    try:
        # ---- the README script (p_cut 1e-2 and the LD file are this fixture's parameters)
        import numpy as np  # noqa: F811
        from gmat.gmatrix import agmat
        from gmat.uvlmm.uvlmm_varcom import wemai_multi_gmat
        from gmat.remma.remma_epiAA import remma_epiAA
        from gmat.remma import annotation_snp_pos
        bed_file = 'plink'
        np.random.seed(1234)
        agmat(bed_file)
        pheno_file = 'pheno'
        ag = np.loadtxt(bed_file + '.agrm0')
        gmat_lst = [ag, ag * ag]
        wemai_multi_gmat(pheno_file, bed_file, gmat_lst, out_file='var_a_axa.txt')
        var_com = np.loadtxt('var_a_axa.txt')
        np.random.seed(4321)
        remma_epiAA(pheno_file, bed_file, gmat_lst, var_com, p_cut=1.0e-2, out_file='epiAA_a_axa')
        res_file = 'epiAA_a_axa'
        annotation_snp_pos(res_file, bed_file, p_cut=1.0e-2, dis=0, ld_file='plink.ld', r2=0.2)
        # ----
        np.testing.assert_allclose(ag, np.load(os.path.join(README, "agrm.npz"))["agrm"], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(var_com, np.loadtxt(os.path.join(README, "var_a_axa.txt")), rtol=1e-6)
        _cmp_table("epiAA_a_axa", os.path.join(README, "epiAA_a_axa"), 2, {2, 3, 4})
        _cmp_table("epiAA_a_axa.anno", os.path.join(README, "epiAA_a_axa.anno"), 14, {14, 15, 16})
        _cmp_table("epiAA_a_axa.anno.ld", os.path.join(README, "epiAA_a_axa.anno.ld"), 14, {14, 15, 16})
    finally:
        os.chdir(cwd)


def test_read_plink_and_impute_match_oracle():
    """gmat.process_plink: the decoded matrix (NaN = missing) and the seeded imputation equal
    the oracle's restatement (pinned to the reference by test_oracle_golden)."""
    from oracle import gmat_oracle as O
    from gmat.process_plink.process_plink import read_plink, impute_geno
    prefix = os.path.join(README, "plink")
    got = read_plink(prefix)
    exp = O.read_plink(prefix)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(exp))
    np.testing.assert_array_equal(np.nan_to_num(got, nan=-1), np.nan_to_num(exp, nan=-1))
    np.random.seed(7)
    a = impute_geno(got)
    np.random.seed(7)
    b = O.impute_geno(exp)
    np.testing.assert_array_equal(a, b)
    assert not np.isnan(a).any()
