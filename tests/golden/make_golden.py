"""Generate the golden fixtures in tests/golden/ by running the REFERENCE GMAT code.

Container-only (needs /root/reference).  The reference is imported through
oracle/ref_shim.py (pandas_plink / cffi / np.int shims); everything it
computes is written here as small data fixtures (inputs and expected outputs), never as
code.  Re-run with:  python tests/golden/make_golden.py

Fixtures ("reference code + its own C decoder in fp64"):
  mouse/   examples/data/mouse (cfg1): agmat/dgmat summaries, REML [A,AxA] (with the
           per-iteration history) and 5-GRM, exact epiAA/AD/DD hit files, a 5,000-pair
           epiAA_pair file, parallel parts, annotation, and the C effect screen.
  tiny/    a 150 x 200 related synthetic cohort (n % 4 == 2, two monomorphic SNPs and one
           all-heterozygous SNP) with full K/D and every testable pair for AA/AD/DD.
           rep*: repeated records (Z != I) REML + epiAA, and wemai_multi_gmat_pred.
  readme/  the README exact-test workflow on a cohort with missing calls and covariates
           (seeded imputation), including the annotation LD filter.
  both:    remma_add / remma_dom result files (``python tests/golden/make_golden.py singles``
           regenerates only these).
"""
import gzip
import hashlib
import json
import logging
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle.ref_shim import import_reference  # noqa: E402
from gmat_amd import synth  # noqa: E402

MOUSE = "/root/reference/examples/data/mouse"


class _Capture(logging.Handler):
    def __init__(self):
        super().__init__()
        self.msgs = []

    def emit(self, record):
        self.msgs.append(record.getMessage())


def _history(msgs):
    out = []
    for m in msgs:
        if m.startswith("Updated variances: "):
            out.append([float(v) for v in m.split(": ", 1)[1].split()])
    return np.array(out)


def _md5(path):
    return hashlib.md5(open(path, "rb").read()).hexdigest()


def _grm_summary(k, path_txt, rng):
    n = k.shape[0]
    ia = rng.integers(0, n, 400)
    ib = rng.integers(0, n, 400)
    return dict(diag=np.diag(k).copy(), row0=k[0].copy(), ia=ia, ib=ib, val=k[ia, ib],
                trace=np.trace(k), total=k.sum(), md5=np.array(_md5(path_txt)))


def mouse(gmat, work, out):
    from gmat.gmatrix import agmat, dgmat_as
    from gmat.uvlmm import wemai_multi_gmat
    from gmat.remma import annotation_snp_pos
    from gmat.remma.remma_epiAA import remma_epiAA, remma_epiAA_pair, remma_epiAA_parallel, remma_epiAA_eff
    from gmat.remma.remma_epiDD import remma_epiDD, remma_epiDD_eff
    from gmat.remma.remma_epiAD import remma_epiAD, remma_epiAD_eff
    os.makedirs(out, exist_ok=True)
    for f in ("plink.bed", "plink.bim", "plink.fam", "pheno"):
        shutil.copy(os.path.join(MOUSE, f), work)
        shutil.copy(os.path.join(MOUSE, f), out)  # input data travels with the fixtures
    bed = os.path.join(work, "plink")
    pheno = os.path.join(work, "pheno")
    rng = np.random.Generator(np.random.PCG64(11))
    a, _ = agmat(bed)
    np.savez(os.path.join(out, "agmat.npz"), **_grm_summary(a, bed + ".agrm0", rng))
    d, _ = dgmat_as(bed)
    np.savez(os.path.join(out, "dgmat_as.npz"), **_grm_summary(d, bed + ".dgrm_as0", rng))
    # agmat with inv=True and the two text formats on a fixed 6x6 corner is covered by tiny/
    cap = _Capture()
    root = logging.getLogger()
    root.addHandler(cap)
    root.setLevel(logging.INFO)
    var2 = wemai_multi_gmat(pheno, bed, [a, a * a], out_file=os.path.join(work, "var2"))
    hist2 = _history(cap.msgs)
    cap.msgs.clear()
    var5 = wemai_multi_gmat(pheno, bed, [a, d, a * a, a * d, d * d], out_file=os.path.join(work, "var5"))
    hist5 = _history(cap.msgs)
    root.removeHandler(cap)
    np.savez(os.path.join(out, "reml.npz"), var2=var2, hist2=hist2, var5=var5, hist5=hist5)
    shutil.copy(os.path.join(work, "var2"), os.path.join(out, "wemai_multi_gmat.var2"))

    g2 = [a, a * a]
    g5 = [a, d, a * a, a * d, d * d]
    remma_epiAA(pheno, bed, g2, var2, p_cut=1e-5, out_file=os.path.join(out, "epiAA_1e-5"))
    remma_epiAA(pheno, bed, g2, var2, p_cut=1e-3, out_file=os.path.join(out, "epiAA_1e-3"))
    remma_epiAD(pheno, bed, g5, var5, p_cut=1e-5, out_file=os.path.join(out, "epiAD_1e-5"))
    remma_epiDD(pheno, bed, g5, var5, p_cut=1e-5, out_file=os.path.join(out, "epiDD_1e-5"))
    for k in (1, 2, 3):
        remma_epiAA_parallel(pheno, bed, g2, var2, [3, k], p_cut=1e-4,
                             out_file=os.path.join(out, "epiAA_par3_1e-4"))
    # fixed pair list (header + 5000 pairs i<j)
    m = sum(1 for _ in open(bed + ".bim"))
    pr = np.random.Generator(np.random.PCG64(5))
    i = pr.integers(0, m - 1, 6000)
    j = pr.integers(0, m, 6000)
    keep = i < j
    pairs = np.column_stack([i[keep], j[keep]])[:5000]
    pair_file = os.path.join(out, "pairs5000")
    np.savetxt(pair_file, pairs, fmt="%d", header="snp_0 snp_1", comments="")
    remma_epiAA_pair(pheno, bed, g2, var2, pair_file, p_cut=1.0, out_file=os.path.join(out, "epiAA_pair5000"))
    annotation_snp_pos(os.path.join(out, "epiAA_1e-3"), bed, p_cut=1e-4, dis=1000000)
    # C effect screen: rows 0..199, fixed var_app so the threshold is known
    rows = list(range(200))
    cwd = os.getcwd()
    os.chdir(work)
    try:
        remma_epiAA_eff(pheno, bed, g2, var2, snp_lst_0=rows, var_app=1470.0, p_cut=1e-2,
                        out_file=os.path.join(out, "epiAA_eff_rows200"))
        remma_epiDD_eff(pheno, bed, g5, var5, snp_lst_0=rows, var_app=490.0, p_cut=1e-2,
                        out_file=os.path.join(out, "epiDD_eff_rows200"))
        remma_epiAD_eff(pheno, bed, g5, var5, snp_lst_0=rows, var_app=960.0, p_cut=1e-2,
                        out_file=os.path.join(out, "epiAD_eff_rows200"))
    finally:
        os.chdir(cwd)


def tiny(gmat, work, out):
    from gmat.gmatrix import agmat, dgmat_as
    from gmat.uvlmm import wemai_multi_gmat
    from gmat.remma.remma_epiAA import remma_epiAA
    from gmat.remma.remma_epiDD import remma_epiDD
    from gmat.remma.remma_epiAD import remma_epiAD
    os.makedirs(out, exist_ok=True)
    n, m = 150, 200
    geno = synth.simulate_genotypes(n, m, seed=3, n_founder=20, n_gen=4, block=40)
    geno[17] = 0          # monomorphic (all hom first allele)
    geno[101] = 2         # monomorphic (all hom second allele)
    geno[150] = 1         # every individual heterozygous: A coding is identically 0
    prefix = os.path.join(out, "tiny")
    synth.write_plink(prefix, geno, seed=3)
    y = synth.simulate_phenotype(geno, seed=4)
    ids = [("F%d" % (i // 10), "I%d" % i) for i in range(n)]
    synth.write_pheno(prefix + ".pheno", ids, y)
    for ext in (".bed", ".bim", ".fam", ".pheno"):
        shutil.copy(prefix + ext, os.path.join(work, "tiny" + ext))
    bed = os.path.join(work, "tiny")
    pheno = bed + ".pheno"
    a, ainv = agmat(bed, inv=True)
    d, _ = dgmat_as(bed)
    agmat(bed, out_fmt="row_col_val")
    agmat(bed, out_fmt="id_id_val")
    # text outputs: md5 + first lines only (the full matrices are in tiny_ref.npz)
    with open(os.path.join(out, "text_outputs.json"), "w") as f:
        json.dump({ext: {"md5": _md5(bed + ext), "head": open(bed + ext).read().splitlines()[:3]}
                   for ext in (".agrm0", ".agrm1", ".agrm2", ".agiv0", ".dgrm_as0")}, f, indent=1)
    cap = _Capture()
    root = logging.getLogger()
    root.addHandler(cap)
    root.setLevel(logging.INFO)
    var = wemai_multi_gmat(pheno, bed, [a, a * a], out_file=os.path.join(work, "var"))
    hist = _history(cap.msgs)
    root.removeHandler(cap)
    np.savez(os.path.join(out, "tiny_ref.npz"), agmat=a, agmat_inv=ainv, dgmat=d, var=var, hist=hist)
    remma_epiAA(pheno, bed, [a, a * a], var, p_cut=1.0, out_file=os.path.join(out, "epiAA_all"))
    remma_epiDD(pheno, bed, [a, a * a], var, p_cut=1.0, out_file=os.path.join(out, "epiDD_all"))
    remma_epiAD(pheno, bed, [a, a * a], var, p_cut=1.0, out_file=os.path.join(out, "epiAD_all"))
    for name in ("epiAA_all", "epiDD_all", "epiAD_all"):
        path = os.path.join(out, name)
        with open(path, "rb") as fi, gzip.open(path + ".gz", "wb", compresslevel=9) as fo:
            fo.write(fi.read())
        os.remove(path)


def singles(gmat, work, out_mouse, out_tiny):
    """Single-SNP tests remma_add / remma_dom (remma_add.py:15-77, remma_dom.py:15-79) on mouse
    ([A, AxA] and the 5-GRM variances) and on tiny (monomorphic SNPs -> NaN statistics)."""
    from gmat.gmatrix import agmat, dgmat_as
    from gmat.remma import remma_add, remma_dom
    for f in ("plink.bed", "plink.bim", "plink.fam", "pheno"):
        shutil.copy(os.path.join(MOUSE, f), work)
    bed = os.path.join(work, "plink")
    pheno = os.path.join(work, "pheno")
    a, _ = agmat(bed)
    d, _ = dgmat_as(bed)
    ref = np.load(os.path.join(out_mouse, "reml.npz"))
    remma_add(pheno, bed, [a, a * a], ref["var2"], out_file=os.path.join(out_mouse, "remma_add"))
    remma_dom(pheno, bed, [a, d, a * a, a * d, d * d], ref["var5"], out_file=os.path.join(out_mouse, "remma_dom"))
    for ext in (".bed", ".bim", ".fam", ".pheno"):
        shutil.copy(os.path.join(out_tiny, "tiny" + ext), os.path.join(work, "tiny" + ext))
    bed = os.path.join(work, "tiny")
    tref = np.load(os.path.join(out_tiny, "tiny_ref.npz"))
    a, d = tref["agmat"], tref["dgmat"]
    remma_add(bed + ".pheno", bed, [a, a * a], tref["var"], out_file=os.path.join(out_tiny, "remma_add"))
    remma_dom(bed + ".pheno", bed, [a, d], tref["var"], out_file=os.path.join(out_tiny, "remma_dom"))


def repeated(gmat, work, out_tiny):
    """Repeated records (Z != I): 1-3 records per individual with a covariate, REML and an
    exact AA scan; and the prediction workflow (wemai_multi_gmat_pred) with 15 genotyped
    individuals lacking records (design_matrix.py:60-113, uvlmm_varcom.py:129-167)."""
    from gmat.uvlmm import wemai_multi_gmat, wemai_multi_gmat_pred
    from gmat.remma.remma_epiAA import remma_epiAA
    for ext in (".bed", ".bim", ".fam"):
        shutil.copy(os.path.join(out_tiny, "tiny" + ext), os.path.join(work, "tiny" + ext))
    bed = os.path.join(work, "tiny")
    tref = np.load(os.path.join(out_tiny, "tiny_ref.npz"))
    a = tref["agmat"]
    ids = [l.split()[:2] for l in open(bed + ".fam")]
    rng = np.random.Generator(np.random.PCG64(8))
    lines, lines_pred = [], []
    skip = set(rng.choice(len(ids), 15, replace=False).tolist())
    base = rng.standard_normal(len(ids))
    for k, (fid, iid) in enumerate(ids):
        for _ in range(int(rng.integers(1, 4))):
            cov = rng.uniform(-1, 1)
            yv = 1.0 + 0.5 * cov + base[k] + 0.7 * rng.standard_normal()
            row = "%s %s 1 %.6f %.6f" % (fid, iid, cov, yv)
            lines.append(row)
            if k not in skip:
                lines_pred.append(row)
    rng.shuffle(lines)  # records need not be grouped or ordered
    with open(os.path.join(out_tiny, "rep.pheno"), "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(out_tiny, "rep_pred.pheno"), "w") as f:
        f.write("\n".join(lines_pred) + "\nF0 I0 1 0.0 NA\n")
    g = [a, a * a]
    var = wemai_multi_gmat(os.path.join(out_tiny, "rep.pheno"), bed, g, out_file=os.path.join(work, "v"))
    remma_epiAA(os.path.join(out_tiny, "rep.pheno"), bed, g, var, p_cut=0.05, out_file=os.path.join(out_tiny, "rep_epiAA"))
    wemai_multi_gmat_pred(os.path.join(out_tiny, "rep_pred.pheno"), bed, g, out_file=os.path.join(work, "pred"))
    np.savez(os.path.join(out_tiny, "rep_ref.npz"), var=var, pred_var=np.loadtxt(os.path.join(work, "pred.var")),
             rand_eff=np.loadtxt(os.path.join(work, "pred.rand_eff")))


def maf_eff(gmat, work, out_mouse):
    """Per-frequency-class effect screens (remma_epi{AA,AD,DD}_maf_eff, C print_out*_maf) on mouse
    rows 0..199: classes computed as the _maf_approx pipelines do, a fixed 111-entry
    denominator table (so the thresholds are known), p_cut 1e-2."""
    from gmat.gmatrix import agmat, dgmat_as
    from gmat.remma.remma_epiAA.remma_epiAA_maf_eff import remma_epiAA_maf_eff
    from gmat.remma.remma_epiAD.remma_epiAD_maf_eff import remma_epiAD_maf_eff
    from gmat.remma.remma_epiDD.remma_epiDD_maf_eff import remma_epiDD_maf_eff
    from gmat.process_plink.process_plink import read_plink
    for f in ("plink.bed", "plink.bim", "plink.fam", "pheno"):
        shutil.copy(os.path.join(MOUSE, f), work)
    bed = os.path.join(work, "plink")
    pheno = os.path.join(work, "pheno")
    a, _ = agmat(bed)
    d, _ = dgmat_as(bed)
    ref = np.load(os.path.join(out_mouse, "reml.npz"))
    snp = read_plink(bed)
    n = snp.shape[0]
    f_aa = 1 - np.sum(snp, axis=0) / (2 * n)
    f_aa[f_aa > 0.5] = 1 - f_aa[f_aa > 0.5]
    f_aa = np.array(list(map(np.longlong, f_aa * 20)), dtype=np.longlong)
    f_d = np.sum(np.absolute(snp - 1.0) < 0.001, axis=0) / n
    f_d[f_d > 0.5] = 1 - f_d[f_d > 0.5]
    f_d = np.array(f_d * 20, dtype=np.longlong)
    f_a = np.sum(snp, axis=0) / (2 * n)
    f_a[f_a > 0.5] = 1 - f_a[f_a > 0.5]
    f_a = np.array(f_a * 20, dtype=np.longlong)
    k = np.arange(111)
    rows = list(range(200))
    g2, g5 = [a, a * a], [a, d, a * a, a * d, d * d]
    cwd = os.getcwd()
    os.chdir(work)
    try:
        remma_epiAA_maf_eff(pheno, bed, g2, ref["var2"], snp_lst_0=rows, freq=f_aa, freq_deno=1470.0 * (0.8 + 0.004 * k),
                            p_cut=1e-2, out_file=os.path.join(out_mouse, "epiAA_maf_eff_rows200"))
        remma_epiDD_maf_eff(pheno, bed, g5, ref["var5"], snp_lst_0=rows, freq=f_d, freq_deno=490.0 * (0.8 + 0.004 * k),
                            p_cut=1e-2, out_file=os.path.join(out_mouse, "epiDD_maf_eff_rows200"))
        remma_epiAD_maf_eff(pheno, bed, g5, ref["var5"], snp_lst_0=rows, freqA=f_a, freqD=f_d,
                            freq_deno=960.0 * (0.8 + 0.004 * k), p_cut=1e-2,
                            out_file=os.path.join(out_mouse, "epiAD_maf_eff_rows200"))
    finally:
        os.chdir(cwd)


def readme(gmat, work, out):
    """The README's exact-test workflow (README.md:94-120): agmat -> np.loadtxt('.agrm0') ->
    wemai_multi_gmat -> remma_epiAA -> annotation_snp_pos (with an LD file), run unchanged on a
    cohort with missing calls (imputation, process_plink.py:12-25) and two covariates besides
    the intercept.  np.random is seeded before each call that imputes (the reference's draws use
    the global state), so the imputed genotypes are reproducible."""
    from gmat.gmatrix import agmat
    from gmat.uvlmm.uvlmm_varcom import wemai_multi_gmat
    from gmat.remma.remma_epiAA import remma_epiAA
    from gmat.remma import annotation_snp_pos
    os.makedirs(out, exist_ok=True)
    n, m = 160, 240
    geno = synth.simulate_genotypes(n, m, seed=21, n_founder=20, n_gen=4, block=40)
    rng = np.random.Generator(np.random.PCG64(22))
    missing = rng.random((m, n)) < 0.03
    prefix = os.path.join(out, "plink")
    synth.write_plink(prefix, geno, missing=missing, seed=21)
    y = synth.simulate_phenotype(geno, seed=23)
    cov = np.column_stack([rng.integers(0, 2, n), rng.uniform(20, 60, n)])
    y = y + 0.5 * cov[:, 0] + 0.02 * cov[:, 1]
    synth.write_pheno(os.path.join(out, "pheno"), [("F%d" % (i // 10), "I%d" % i) for i in range(n)], y, covar=cov)
    # PLINK --r2 layout: CHR_A BP_A SNP_A CHR_B BP_B SNP_B R2 (annotation.py:57-64 reads 2, 5, -1)
    bim = [l.split() for l in open(prefix + ".bim")]
    with open(os.path.join(out, "plink.ld"), "w") as f:
        f.write(" CHR_A BP_A SNP_A CHR_B BP_B SNP_B R2\n")
        for a in range(0, m - 1, 2):
            for b in (a + 1, a + 7):
                if b < m:
                    f.write(" %s %s %s %s %s %s %.6f\n" % (bim[a][0], bim[a][3], bim[a][1], bim[b][0], bim[b][3],
                                                           bim[b][1], rng.uniform(0, 0.5)))
    for name in ("plink.bed", "plink.bim", "plink.fam", "pheno", "plink.ld"):
        shutil.copy(os.path.join(out, name), work)
    cwd = os.getcwd()
    os.chdir(work)
    try:
        bed_file = "plink"
        np.random.seed(1234)
        agmat(bed_file)
        pheno_file = "pheno"
        ag = np.loadtxt(bed_file + ".agrm0")
        gmat_lst = [ag, ag * ag]
        wemai_multi_gmat(pheno_file, bed_file, gmat_lst, out_file="var_a_axa.txt")
        var_com = np.loadtxt("var_a_axa.txt")
        np.random.seed(4321)
        remma_epiAA(pheno_file, bed_file, gmat_lst, var_com, p_cut=1.0e-2, out_file="epiAA_a_axa")
        annotation_snp_pos("epiAA_a_axa", bed_file, p_cut=1.0e-2, dis=0, ld_file="plink.ld", r2=0.2)
        np.savez(os.path.join(out, "agrm.npz"), agrm=ag)
        for name in ("var_a_axa.txt", "epiAA_a_axa", "epiAA_a_axa.anno", "epiAA_a_axa.anno.ld"):
            shutil.copy(name, os.path.join(out, name))
    finally:
        os.chdir(cwd)


def main():
    gmat = import_reference()
    logging.getLogger().setLevel(logging.WARNING)
    what = sys.argv[1:] or ["tiny", "mouse", "singles", "repeated", "maf", "readme"]
    if "tiny" in what:
        with tempfile.TemporaryDirectory() as work:
            tiny(gmat, work, os.path.join(HERE, "tiny"))
    if "mouse" in what:
        with tempfile.TemporaryDirectory() as work:
            mouse(gmat, work, os.path.join(HERE, "mouse"))
    if "singles" in what:
        with tempfile.TemporaryDirectory() as work:
            singles(gmat, work, os.path.join(HERE, "mouse"), os.path.join(HERE, "tiny"))
    if "maf" in what:
        with tempfile.TemporaryDirectory() as work:
            maf_eff(gmat, work, os.path.join(HERE, "mouse"))
    if "repeated" in what:
        with tempfile.TemporaryDirectory() as work:
            repeated(gmat, work, os.path.join(HERE, "tiny"))
    if "readme" in what:
        with tempfile.TemporaryDirectory() as work:
            readme(gmat, work, os.path.join(HERE, "readme"))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
