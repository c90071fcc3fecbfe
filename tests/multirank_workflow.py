"""A reference-style user script on the mouse example (README.md:94-210 call forms, through
``import gmat``), run by tests/test_gpu_multirank.py unchanged as 1 rank and as N ranks of one job
(``python -m gmat_amd.launch --gpus N``): GRMs, REML, the exact scans AA / AD / DD, a
triangle-folded part, a pair list, the effect screen, a random-pair approximate test and the
annotation.  Every output file lands in the working directory given as argv[1].

    python tests/multirank_workflow.py OUT_DIR GOLDEN_MOUSE_DIR
"""
import os
import shutil
import sys

import numpy as np

out_dir, mouse = sys.argv[1], sys.argv[2]
for f in ("plink.bed", "plink.bim", "plink.fam", "pheno", "pairs5000"):
    if int(os.environ.get("RANK", "0")) == 0:
        shutil.copy(os.path.join(mouse, f), out_dir)
os.chdir(out_dir)

import gmat  # noqa: E402,F401
from gmat.gmatrix import agmat, dgmat_as  # noqa: E402
from gmat.uvlmm.uvlmm_varcom import wemai_multi_gmat  # noqa: E402
from gmat.remma.remma_epiAA import remma_epiAA, remma_epiAA_parallel, remma_epiAA_pair  # noqa: E402
from gmat.remma.remma_epiAA import remma_epiAA_eff, remma_epiAA_approx  # noqa: E402
from gmat.remma.remma_epiAD import remma_epiAD  # noqa: E402
from gmat.remma.remma_epiDD import remma_epiDD  # noqa: E402
from gmat.remma import annotation_snp_pos  # noqa: E402

bed_file, pheno_file = "plink", "pheno"
np.random.seed(1234)
ka = agmat(bed_file)[0]
kd = dgmat_as(bed_file)[0]
ag = np.loadtxt(bed_file + ".agrm0")  # the README reads the file rank 0 wrote back
assert np.array_equal(ag, ka)
g2 = [ka, ka * ka]
g5 = [ka, kd, ka * ka, ka * kd, kd * kd]
ref = np.load(os.path.join(mouse, "reml.npz"))
var2 = wemai_multi_gmat(pheno_file, bed_file, g2, out_file="var_a_axa.txt")
assert np.array_equal(var2, np.loadtxt("var_a_axa.txt"))
remma_epiAA(pheno_file, bed_file, g2, ref["var2"], p_cut=1e-5, out_file="epiAA_1e-5")
remma_epiAA(pheno_file, bed_file, g2, ref["var2"], p_cut=1e-3, out_file="epiAA_1e-3")
remma_epiAD(pheno_file, bed_file, g5, ref["var5"], p_cut=1e-5, out_file="epiAD_1e-5")
remma_epiDD(pheno_file, bed_file, g5, ref["var5"], p_cut=1e-5, out_file="epiDD_1e-5")
for k in (1, 2, 3):
    remma_epiAA_parallel(pheno_file, bed_file, g2, ref["var2"], [3, k], p_cut=1e-4, out_file="epiAA_par3_1e-4")
remma_epiAA_pair(pheno_file, bed_file, g2, ref["var2"], "pairs5000", p_cut=1.0, out_file="epiAA_pair5000")
remma_epiAA(pheno_file, bed_file, g2, ref["var2"], snp_lst_0=[700, 3, 3, 1200, 5], p_cut=1e-2, out_file="epiAA_rows")
remma_epiAA_eff(pheno_file, bed_file, g2, ref["var2"], snp_lst_0=list(range(200)), var_app=1470.0, p_cut=1e-2,
                out_file="epiAA_eff_rows200")
remma_epiAA_approx(pheno_file, bed_file, g2, ref["var2"], p_cut=1e-4, num_random_pair=20000, out_file="epiAA_approx",
                   seed=11)
annotation_snp_pos("epiAA_1e-3", bed_file, p_cut=1e-4, dis=1000000)
print("workflow done on rank %s" % os.environ.get("RANK", "0"), flush=True)
