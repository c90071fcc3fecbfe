"""Headline benchmark: exhaustive exact remma_epiAA on a synthetic 2,000 x 50,000 cohort.

BASELINE.json metric: "SNP-pairs tested/sec (whole node) + GRM GFLOP/s".
One step = one full epiAA scan of the m(m-1)/2 = 1,249,975,000 SNP pairs (configs[2];
with --gpus N the same cohort is sharded over N ranks = configs[3], strong scaling).
The genotype panel, P and Py are resident in HBM before the timed region; the step
includes the screen, the exact fp64 refine of the candidates and the hit collection.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Rank 0 prints one JSON line.  Extra objects: roofline (the int8 screen kernel, measured
with HIP events inside libgmat_hip on its launch stream), cpu_baseline (the oracle's
numpy restatement of the reference per-row loop on a bounded row sample, rank 0, N=1),
grm (configs[1]: agmat GRM on 2,000 x 20,000, GFLOP/s dense-equivalent 2n^2m).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "SNP-pairs tested/sec (whole node) + GRM GFLOP/s, mouse-sized cohort"
INT8_PEAK_TOPS = 5000.0  # MI355X dense int8 MFMA (2x the 2.5 PF dense bf16), MI355X_MICROARCH.md
MX_PEAK_TFLOPS = 10000.0  # dense block-scaled fp6/fp4 MFMA (4x bf16 per clock), MI355X_MICROARCH.md
LDS_DMA_PEAK_TBPS = 6.4  # chip-wide L2/MALL -> LDS rate of LDS-DMA with every CU streaming, MI355X_MICROARCH.md
FP64_PEAK_TFLOPS = 78.6  # dense fp64 MFMA, MI355X_MICROARCH.md


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def covariate_design(n, seed, y0):
    """[1, binary, integer 90-129, binary] (the reference's example pheno layout) and the phenotype
    with covariate effects (shared by --covariates and the covariates leg)."""
    rng = np.random.Generator(np.random.PCG64(seed + 9))
    x = np.column_stack([np.ones(n), rng.integers(0, 2, n), rng.integers(90, 130, n), rng.integers(0, 2, n)])
    return x.astype(float), y0 + 0.3 * x[:, 1] + 0.01 * x[:, 2] - 0.2 * x[:, 3]


def build_inputs(n, m, seed, var, rank, ws, covariates=False):
    """Cohort (deterministic, generated shard by shard: rank r makes only its SNP range), the
    packed shards all-gathered over RCCL, P / Py computed on rank 0 and broadcast."""
    from gmat_amd import dist, synth
    from gmat_amd import _native as N
    nb = (n + 3) // 4
    t0 = time.time()
    lo, hi = dist.snp_shard(m, rank, ws)
    shard, n_bad = synth.simulate_genotype_shard(n, m, lo, hi, seed=seed)  # (hi - lo, n)
    if dist.allreduce_sum(n_bad) > 0:  # the full generator re-draws (near-)monomorphic SNPs
        shard = synth.simulate_genotypes(n, m, seed=seed)[lo:hi]
    local = np.frombuffer(synth.pack_bed(shard)[3:], dtype=np.uint8).reshape(hi - lo, nb)
    body = dist.allgather_packed(local, m, nb)
    geno = shard if ws == 1 else None
    log("cohort %d x %d: shard [%d, %d) generated, panel all-gathered in %.1f s" % (n, m, lo, hi, time.time() - t0))
    from gmat_amd.plink import Geno
    g = Geno(body=body, n_id=n, n_snp=m)
    pvp = py = ka = y = None
    if rank == 0:
        pvp, py, ka, y = _rank0_inputs(g, n, seed, var, covariates)
    pvp = dist.broadcast_array(pvp, 0, shape=(n, n))
    py = dist.broadcast_array(py, 0, shape=(n,))
    return geno, g, pvp, py, ka, y


def _rank0_inputs(g, n, seed, var, covariates):
    """GRM, simulated phenotype and P / Py of the cohort (rank 0: the drop-in API as one process)."""
    import ctypes
    from gmat_amd import dist
    from gmat_amd import _native as N
    with dist.local():
        lib = N.ensure_device()
        ka = np.empty((n, n))
        sc = ctypes.c_double()
        N.check(lib.gmat_grm(g.handle, 0, 0.001, N.ptr(ka), ctypes.byref(sc)), "gmat_grm")
        rng = np.random.Generator(np.random.PCG64(seed + 1))
        y = np.ones(n)
        for k, s in ((ka, var[0]), (ka * ka, var[1])):
            y += np.sqrt(s) * (np.linalg.cholesky(k + 1e-4 * np.eye(n)) @ rng.standard_normal(n))
        y += np.sqrt(var[2]) * rng.standard_normal(n)
        from scipy.sparse import identity
        from gmat_amd.uvlmm.uvlmm_varcom import projection
        x = np.ones((n, 1))
        if covariates:
            x, y = covariate_design(n, seed, y)
        pvp, py = projection(y, x, identity(n, format="csr"), [ka, ka * ka], var)
    return pvp, py, ka, y


def cpu_baseline(geno, pvp, py, budget_s):
    """The oracle's restatement of _remma_epiAA's per-row loop (remma_epiAA.py:71-82, numpy
    fp64 + the host BLAS), timed on stratified rows until `budget_s` elapses.  Returns the
    baseline record plus the rows used and the oracle's hits on them (the parity check)."""
    from oracle import gmat_oracle as O  # checker / CPU baseline only
    snp = np.ascontiguousarray(geno.T, dtype=np.float64)
    m = snp.shape[1]
    order = np.linspace(0, m - 2, 64).astype(np.int64)
    rng = np.random.default_rng(0)
    rng.shuffle(order)
    pairs, t0, used, hits = 0, time.perf_counter(), [], []
    for i in order:
        hits.append(O.epi_scan("AA", snp, pvp, py.reshape(-1, 1), snp_lst_0=[int(i)], p_cut=1e-5))
        pairs += m - 1 - int(i)
        used.append(int(i))
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    rec = {"value": pairs / dt, "unit": "SNP-pairs/s", "cores": cores, "kind": "port",
           "sample": "%d stratified rows of the same 2000x50000 cohort (%d pairs, %.1f s), numpy/BLAS fp64 "
                     "restatement of remma_epiAA.py:71-82" % (len(used), pairs, dt)}
    exp = np.concatenate(hits) if hits else np.zeros((0, 5))
    return rec, np.array(used, dtype=np.int64), exp


def parity_check(plan, rows, exp, p_cut):
    """GPU hits on the oracle's rows (every screen level the plan has) against the oracle's
    exact fp64 hits: identical (i, j) sets, eff / chi / p within 1e-8 relative."""
    order = np.argsort(rows)
    rows = rows[order]
    exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))] if exp.size else exp
    out = {"rows": int(rows.size), "oracle_hits": int(exp.shape[0]), "levels": {}}
    ok = True
    for ns, name in ((0, "auto"), (-1, "mx"), (1, "int8x1")):
        hi, hj, eff, var, chi, p = plan.scan("AA", rows, p_cut, n_slice=ns)
        same = hi.size == exp.shape[0] and np.array_equal(np.column_stack([hi, hj]), exp[:, :2].astype(np.int64))
        err = 0.0
        if same and hi.size:
            got = np.column_stack([eff, chi, p])
            err = float(np.max(np.abs(got - exp[:, 2:]) / np.maximum(np.abs(exp[:, 2:]), 1e-300)))
        lev_ok = bool(same and err <= 1e-8)
        out["levels"][name] = {"hits": int(hi.size), "identical_pairs": bool(same), "max_rel_err": err,
                               "screen_level": int(plan.stats()["n_slice"])}
        ok = ok and lev_ok
    out["identical"] = ok
    return out


EXHAUSTIVE_HITS = os.path.join(REPO, "tests", "golden", "cfg3_exhaustive_hits_AA_2000x50000.npz")
FULL_TRIANGLE_RECORD = "profiles/round5_full_triangle_AA_2000x50000.json"


def full_triangle_check(g, pvp, py, hits, p_cut, live=None):
    """The timed step's hits (merged over the ranks) against the EXHAUSTIVE scan of the same cohort:
    every one of the 1,249,975,000 pairs refined in fp64 with no screen (gmat_epi_scan level
    GMAT_SCREEN_NONE, the reference's computation remma_epiAA.py:71-82), recorded by
    tools/full_triangle.py (FULL_TRIANGLE_RECORD; hit set in tests/golden) or, with
    --full-triangle, recomputed in this run (`live`).  Identical (i, j) sets and byte-identical
    eff / var / chi / p are required; a cohort fingerprint (per-SNP counts, P, Py) guards the record."""
    from tools.full_triangle import cohort_fingerprint
    out = {"source": "live exhaustive scan in this run" if live is not None else FULL_TRIANGLE_RECORD}
    if live is not None:
        ref = live
    else:
        if not os.path.exists(EXHAUSTIVE_HITS):
            return dict(out, checked=False, reason="no recorded exhaustive hit set")
        d = np.load(EXHAUSTIVE_HITS)
        if bytes(d["fingerprint"]).hex() != cohort_fingerprint(g, pvp, py) or float(d["p_cut"][0]) != p_cut:
            return dict(out, checked=False, reason="recorded hit set is for another cohort / p_cut")
        ref = (d["i"].astype(np.int64), d["j"].astype(np.int64), d["eff"], d["var"], d["chi"], d["p"])
    a = set(zip(hits[0].tolist(), hits[1].tolist()))
    b = set(zip(ref[0].tolist(), ref[1].tolist()))
    sd = len(a ^ b)
    same = sd == 0 and all(np.array_equal(np.asarray(x).view(np.uint64), np.asarray(y).view(np.uint64))
                           for x, y in zip(hits[2:], ref[2:]))
    return dict(out, checked=True, exhaustive_hits=len(b), step_hits=len(a), symmetric_difference=sd,
                values_byte_identical=bool(same), identical=bool(sd == 0 and same))


def exhaustive_live(plan, rows, p_cut, lib):
    """This rank's rows refined with no screen (about 113 s for the whole configs[2] triangle on one
    MI355X); progress on stderr."""
    from gmat_amd import _native as N
    parts, t0 = [], time.perf_counter()
    for k in range(0, rows.size, 2000):
        parts.append(plan.scan("AA", rows[k:k + 2000], p_cut, n_slice=N.GMAT_SCREEN_NONE))
        log("exhaustive: %d / %d rows, %.0f s" % (min(k + 2000, rows.size), rows.size, time.perf_counter() - t0))
    return tuple(np.concatenate([p[t] for p in parts]) for t in range(6)), time.perf_counter() - t0


def grm_bench(n, m_grm, seed, reps=5):
    """configs[1] GRM: agmat product on the block-scaled fp4 MFMA (2-bit fragment images + SYRK, exact
    integer products), product time from HIP events."""
    import ctypes
    from gmat_amd import _native as N, synth
    from gmat_amd.plink import Geno
    lib = N.ensure_device()
    # full-sib families of five in the last generation: A and A x A distinct from the identity, so the
    # configs[1] REML below is identifiable and converges
    geno = synth.simulate_genotypes(n, m_grm, seed=seed + 11, family_size=5)
    body = np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8)
    g = Geno(body=body, n_id=n, n_snp=m_grm)
    k = np.empty((n, n))
    sc = ctypes.c_double()
    st = np.zeros(4)
    times = []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        N.check(lib.gmat_grm(g.handle, 0, 0.001, N.ptr(k), ctypes.byref(sc)), "gmat_grm")
        wall = time.perf_counter() - t0
        N.check(lib.gmat_grm_stats(N.ptr(st)), "gmat_grm_stats")
        if r:
            times.append((st[0], wall))
    g.close()
    grm_bench.last_k = k
    kern = float(np.median([t[0] for t in times]))
    wall = float(np.median([t[1] for t in times]))
    flop = 2.0 * n * n * m_grm
    return {"config": "configs[1]: agmat GRM %d x %d" % (n, m_grm), "gflops_kernel": flop / kern / 1e9,
            "gflops_end_to_end": flop / wall / 1e9, "kernel_ms": kern * 1e3, "end_to_end_ms": wall * 1e3,
            "flop_convention": "dense-equivalent 2 n^2 m", "mfma": "fp4 block-scaled (dosage/2 in e2m1, scale 2)",
            "ops_issued": float(st[1]), "mx_tops": st[1] / kern / 1e12,
            "mx_frac_of_peak": st[1] / kern / 1e12 / MX_PEAK_TFLOPS,
            "int8_equiv_frac_of_peak": st[1] / kern / 1e12 / INT8_PEAK_TOPS,
            "kernel_covers": "the 2-bit image transpose + the SYRK (the centring epilogue and row sums are in "
                             "device_ms_all_kernels)",
            "device_ms_all_kernels": float(st[3]) * 1e3}


def reml_bench(k, seed):
    """configs[1] REML: 2-GRM ([A, AxA] + residual) weighted EM-AI REML at n = 2,000 on the
    device (gmat_reml), synthetic phenotype with (0.4, 0.2, 0.4); seconds per iteration from the
    library's own clock (every iteration ends in a host sync)."""
    from gmat_amd import _native as N
    from gmat_amd.uvlmm.uvlmm_varcom import _wemai_multi_gmat
    from scipy.sparse import identity
    lib = N.ensure_device()
    n = k.shape[0]
    rng = np.random.Generator(np.random.PCG64(seed + 3))
    kk = k * k
    y = np.ones(n)
    for g, s_ in ((k, 0.4), (kk, 0.2)):
        y += np.sqrt(s_) * (np.linalg.cholesky(g + 1e-4 * np.eye(n)) @ rng.standard_normal(n))
    y += np.sqrt(0.4) * rng.standard_normal(n)
    t0 = time.perf_counter()
    var = _wemai_multi_gmat(y, np.ones((n, 1)), identity(n, format="csr"), [k, kk])
    wall = time.perf_counter() - t0
    st = np.zeros(4)
    N.check(lib.gmat_reml_stats(N.ptr(st)), "gmat_reml_stats")
    flop = st[3]
    return {"config": "configs[1]: 2-GRM REML [A, AxA] n=%d, full-sib families of 5, simulated (0.4, 0.2, 0.4)" % n,
            "iters": int(st[1]), "converged": bool(int(st[1]) < 200),
            "ms_per_iter": st[2] * 1e3, "wall_s": wall, "var": [float(v) for v in var],
            "fp64_tflops": flop / st[2] / 1e12 if st[2] > 0 else None,
            "frac": flop / st[2] / 1e12 / FP64_PEAK_TFLOPS if st[2] > 0 else None,
            "flop_convention": "n^3/3 potrf + 2n^3/3 inverse + 2n^2(2c+1) per iteration"}


def e2e_bench(geno, ka, y, var, p_cut, hits_step, reps=5):
    """User-facing remma_epiAA end to end (SURVEY.md 8(b) signature): .bed/.bim/.fam/pheno on
    disk -> design matrix -> P, Py on the device -> genotype decode -> plan (certificates)
    -> exhaustive scan -> hits file.  Same cohort and hits as the timed step.  `reps` calls, the
    median wall time and the median of each phase (remma._scan.LAST_PHASES)."""
    import tempfile
    from gmat_amd import synth
    from gmat_amd.remma import remma_epiAA
    from gmat_amd.remma import _scan
    n = geno.shape[1]
    walls, phases = [], []
    with tempfile.TemporaryDirectory() as d:
        prefix = os.path.join(d, "c")
        synth.write_plink(prefix, geno)
        synth.write_pheno(prefix + ".pheno", [("F%d" % (i // 10), "I%d" % i) for i in range(n)], y)
        for _ in range(reps):
            t0 = time.perf_counter()
            remma_epiAA(prefix + ".pheno", prefix, [ka, ka * ka], var, p_cut=p_cut, out_file=prefix + ".epiAA")
            walls.append(time.perf_counter() - t0)
            ph = dict(_scan.LAST_PHASES)
            ph["design_and_other"] = walls[-1] - sum(ph.values())
            phases.append(ph)
        with open(prefix + ".epiAA") as f:
            n_hits = sum(1 for _ in f) - 1
    return {"wall_s": float(np.median(walls)), "wall_s_all": walls, "hits": n_hits,
            "hits_match_step": bool(n_hits == hits_step),
            "phases_s_median": {k: float(np.median([p[k] for p in phases])) for k in phases[0]},
            "what": "remma_epiAA(pheno, bed, [A, AxA], var, p_cut) from files to the hits file, median of %d" % reps}


def covariate_bench(g, ka, y0, n, m, p_cut, seed, steps, ms_intercept):
    """configs[2] with intercept + 3 covariates (binary, integer-valued, binary: the layout of the
    reference's example pheno): P gains three null directions besides 1; the plan certifies the
    prefilter with them (prefilter_cov_kernel) and keeps the low-rank screen.  Whole-scan time."""
    from gmat_amd import _native as N
    from gmat_amd.remma._scan import EpiPlan
    from gmat_amd.uvlmm.uvlmm_varcom import projection
    from scipy.sparse import identity
    lib = N.ensure_device()
    x, y = covariate_design(n, seed, y0)
    pvp, py = projection(y, x, identity(n, format="csr"), [ka, ka * ka], [0.4, 0.2, 0.4])
    rows = np.arange(m - 1, dtype=np.int64)
    t0 = time.perf_counter()
    plan = EpiPlan(g, pvp, py)
    t_plan = time.perf_counter() - t0
    plan.scan("AA", rows, p_cut)
    lib.gmat_device_synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        res = plan.scan("AA", rows, p_cut)
    lib.gmat_device_synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    st = plan.stats()
    out = {"config": "configs[2] cohort, X = [1, binary, integer 90-129, binary]", "ms_per_step": ms,
           "pairs_per_s": m * (m - 1) / 2 / ms * 1e3, "ratio_to_intercept_only": ms / ms_intercept,
           "hits": int(res[0].size), "candidates": st["candidates"], "screen_level": int(st["n_slice"]),
           "covariate_directions": int(plan.setup_stats()["covariate_directions"]), "plan_create_s": t_plan,
           "lowrank_rank": plan.lowrank_rank()}
    plan.close()
    return out


def eff_cpu_baseline(geno, py, cut, budget_s):
    """The C++/OpenMP restatement of _remma_epi_eff_cpu.c (oracle/eff_cpu.cpp, bit-identical to
    the reference's C) timed on the box's host cores on stratified rows of the same cohort."""
    from oracle import gmat_oracle as O  # checker / CPU baseline only
    from gmat_amd import synth
    m, n = geno.shape
    body = synth.pack_bed(geno)[3:]
    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    # two probe calls separate the per-call cost (decode + centring, as the reference's call pays
    # it) from the per-pair rate, which sizes the sample to about budget_s of pair work
    t = []
    for kp in (8, 40):
        probe = np.linspace(0, m - 2, kp).astype(np.int64)
        t0 = time.perf_counter()
        O.eff_screen_c("AA", body, n, m, probe, py, [cut], threads=threads)
        t.append((float(np.sum(m - 1 - probe)), time.perf_counter() - t0))
    # the difference of the two probes is noisy when the per-call decode dominates them: bound the
    # per-pair cost below by a quarter of the larger probe's average (sample <= 4 x budget_s)
    per_pair = max((t[1][1] - t[0][1]) / (t[1][0] - t[0][0]), t[1][1] / t[1][0] / 4.0)
    k = int(min(m - 1, max(8, budget_s / per_pair / (m / 2))))
    rows = np.linspace(0, m - 2, k).astype(np.int64)
    t0 = time.perf_counter()
    O.eff_screen_c("AA", body, n, m, rows, py, [cut], threads=threads)
    dt = time.perf_counter() - t0
    pairs, used = int(np.sum(m - 1 - rows)), rows.size
    return {"value": pairs / dt, "unit": "SNP-pairs/s", "cores": threads, "kind": "port",
            "sample": "%d stratified rows of the 2000x50000 cohort (%d pairs, %.1f s incl. decode), C++/OpenMP "
                      "restatement of _remma_epi_eff_cpu.c:61-137 (oracle/eff_cpu.cpp)" % (used, pairs, dt)}


def eff_bench(g, pvp, py, plan, n, m, p_cut, seed, geno=None, cpu_budget=10.0):
    """Effect-only screen (the remma_epiAA_eff_cpu replacement) over the
    same cohort, threshold from the exact variance median of 20,000 random pairs as
    remma_epiAA_approx does.  Algorithmic 2n flop per pair; f64 MFMA roof."""
    import ctypes
    import tempfile
    from scipy.stats import chi2
    from gmat_amd import _native as N
    lib = N.ensure_device()
    rng = np.random.Generator(np.random.PCG64(seed + 5))
    i = rng.integers(0, m - 1, 40000)
    j = rng.integers(0, m, 40000)
    keep = i < j
    pr = np.column_stack([i[keep], j[keep]])[:20000]
    _, var, _, _ = plan.pairs("AA", pr)
    eff_cut = np.array([np.sqrt(chi2.isf(p_cut, 1) * np.median(var))])
    rows = np.arange(m - 1, dtype=np.int64)
    pyn = N.f64(py)
    nh = ctypes.c_int64()
    st = np.zeros(4)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "eff").encode()
        t0 = time.perf_counter()
        N.check(lib.gmat_eff_scan(g.handle, N.GMAT_AA, N.ptr(pyn), N.ptr(rows), rows.size, N.ptr(eff_cut), None, None,
                                  out, ctypes.byref(nh)), "gmat_eff_scan")
        wall = time.perf_counter() - t0
    N.check(lib.gmat_eff_stats(N.ptr(st)), "gmat_eff_stats")
    pairs = st[0]
    log("effect screen cpu baseline")
    cpu = eff_cpu_baseline(geno, py, float(eff_cut[0]), cpu_budget) if geno is not None else None
    return {"config": "remma_epiAA_eff over all %d pairs, eff_cut from the median var (p_cut=%g)" % (pairs, p_cut),
            "pairs_per_s_device": pairs / st[2], "pairs_per_s_end_to_end": pairs / wall, "device_s": st[2],
            "text_s": st[3], "hits": int(nh.value),
            "algorithmic_tflops": pairs * 2.0 * n / st[2] / 1e12,
            "flop_convention": "2n per pair (SURVEY 8(d)); computed as 2 int8 slices (4n int8 ops) + exact fp64 "
                               "recompute of the candidates",
            "cpu_baseline": cpu}


def split_emulation(plan, m, p_cut, step_ms, hits_step, lib, ways=(2, 4, 8), reps=5, kind="AA"):
    """configs[3] rehearsed on one GPU: each part of the multi-GPU split (dist.rank_rows: part k of
    the reference's folded parallel=[N,k] rows, remma_epiAA.py:125-139) timed serially on this GPU
    -- what one rank of an N-GPU run computes between its barriers.  A part is timed as the step is:
    one untimed scan, then `reps` scans back to back between two device synchronisations, the mean
    (round 4 took the best of two single scans).  Reports per-part ms, the max / mean imbalance and
    the projected N-GPU step (slowest part; the hit gather is a few hundred KB), and checks that the
    parts' hits add up to the 1-GPU step's."""
    from gmat_amd import dist
    out = {}
    for N in ways:
        ms, hits, pairs = [], 0, []
        for k in range(N):
            rows = dist.rank_rows(kind, m, k, N)
            plan.scan(kind, rows, p_cut)
            lib.gmat_device_synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                res = plan.scan(kind, rows, p_cut)
                plan.stats()  # the step's per-scan bookkeeping
            lib.gmat_device_synchronize()
            ms.append((time.perf_counter() - t0) * 1e3 / reps)
            hits += int(res[0].size)
            pairs.append(float(rows.size * m) if kind == "AD" else float(np.sum(m - 1 - rows)))
        mean = float(np.mean(ms))
        out["%d" % N] = {"part_ms": [round(x, 3) for x in ms], "max_over_mean": max(ms) / mean,
                         "pairs_max_over_mean": max(pairs) / float(np.mean(pairs)),
                         "projected_step_ms": max(ms), "projected_speedup": step_ms / max(ms),
                         "projected_efficiency": step_ms / max(ms) / N, "hits_sum": hits,
                         "hits_match_step": bool(hits == hits_step)}
    return out


def cfg5_leg(n, m, p_cut, seed, reml_iters, rank, ws, backend, family_size=None, reps=3, split=True):
    """BASELINE configs[4]: synthetic related 5,000 x 100,000 cohort (60 founders, 6
    generations of random mating; `family_size`: the last generation in full-sib families instead),
    5-GRM model [A, D, AxA, AxD, DxD]: GRMs (agmat / dgmat_as products), weighted EM-AI REML
    (uvlmm_varcom.py:41-99, up to reml_iters iterations or convergence), P / Py from the REML
    ESTIMATE (as remma_epiAD / remma_epiDD get var_com from wemai_multi_gmat in the reference
    workflow), then the exhaustive epiDD (j > i) and epiAD (every ordered pair, i == j included)
    scans at p_cut, rows sharded over the ranks like configs[3] (GRM and REML on rank 0).  Each scan:
    one untimed full scan (codings and buffers at the timed size), then `reps` timed scans, median
    reported.  On one GPU (`split`), each kind's 2 / 4 / 8-way split (dist.rank_rows: the reference's
    folded parallel=[N, k] rows, remma_epiDD.py / remma_epiAD.py:134-140) is rehearsed part by part, as
    configs[3]'s.  Returns the record on rank 0.
    The REML does not meet the reference's stopping rule here (gradient norm < 1e-6): the epistatic
    kernels are near-collinear at this size (asymptotic standard errors 10-48x the simulated AxA / AxD /
    DxD variances, tools/cfg5_identifiability.py), so the pure AI step leaves the positive orthant and
    nearly every iteration needs an EM weight > 0; 0 of 48 phenotype draws converge within 200
    iterations (profiles/round5_cfg5_reml_probe.txt).  The reference's loop returns its 200th iterate
    then, and so does this one (its iterates match the oracle's: tests/test_gpu_cfg5.py)."""
    from gmat_amd import dist, synth
    from gmat_amd import _native as N
    from gmat_amd.plink import Geno
    lib = N.ensure_device()
    nb = (n + 3) // 4
    t0 = time.time()
    lo, hi = dist.snp_shard(m, rank, ws)
    shard, n_bad = synth.simulate_genotype_shard(n, m, lo, hi, seed=seed, family_size=family_size)
    if dist.allreduce_sum(n_bad) > 0:
        shard = synth.simulate_genotypes(n, m, seed=seed, family_size=family_size)[lo:hi]
    local = np.frombuffer(synth.pack_bed(shard)[3:], dtype=np.uint8).reshape(hi - lo, nb)
    del shard
    g = Geno(body=dist.allgather_packed(local, m, nb), n_id=n, n_snp=m)
    t_cohort = time.time() - t0
    log("cfg5 cohort %d x %d in %.1f s" % (n, m, t_cohort))
    var = np.array([0.3, 0.1, 0.1, 0.05, 0.05, 0.4])
    out = {"workload": "configs[4]: 5-GRM REML + exhaustive epiDD / epiAD, %d ind x %d SNP (%s), p_cut=%g"
                       % (n, m, "full-sib families of %d" % family_size if family_size else "random mating", p_cut),
           "n_gpus": ws,
           "parallelism": "scan rows folded over %d rank(s), backend %s; GRM and REML on rank 0" % (ws, backend or "single"),
           "cohort_s": t_cohort}
    pvp = py = None
    if rank == 0:
        pvp, py = _cfg5_rank0(g, n, m, seed, var, reml_iters, out)
    pvp = dist.broadcast_array(pvp, 0, shape=(n, n))
    py = dist.broadcast_array(py, 0, shape=(n,))
    t1 = time.perf_counter()
    plan = dist.shared_plan(g, pvp, py)  # spectral state computed on rank 0, imported by the others
    out["plan_create_s"] = time.perf_counter() - t1
    out["setup"] = plan.setup_stats()
    out["lowrank_rank"] = plan.lowrank_rank()
    total = t_all = 0.0
    for kind in ("DD", "AD"):
        rows = dist.rank_rows(kind, m, rank, ws)
        t1 = time.perf_counter()
        plan.scan(kind, rows, p_cut)  # codings (side vectors) and scan buffers at the timed size, untimed
        lib.gmat_device_synchronize()
        t_first = time.perf_counter() - t1
        times = []
        for _ in range(reps):
            dist.barrier()
            t1 = time.perf_counter()
            res = plan.scan(kind, rows, p_cut)
            lib.gmat_device_synchronize()
            dist.barrier()
            times.append(dist.allreduce_max(time.perf_counter() - t1))
        dt = float(np.median(times))
        pairs = float(m) * (m - 1) / 2 if kind == "DD" else float(m) * m
        st = plan.stats()
        out["epi" + kind] = {"pairs": pairs, "s": dt, "s_all": times, "first_scan_s": t_first, "pairs_per_s": pairs / dt,
                             "hits": int(dist.allreduce_sum(res[0].size)),
                             "candidates": int(dist.allreduce_sum(st["candidates"])), "screen_level": int(st["n_slice"])}
        total += pairs
        t_all += dt
    out["pairs_per_s"] = total / t_all
    if split and ws == 1:
        log("configs[4] split rehearsed part by part")
        out["split_rehearsal"] = {kind: split_emulation(plan, m, p_cut, out["epi" + kind]["s"] * 1e3,
                                                        out["epi" + kind]["hits"], lib, reps=1, kind=kind)
                                  for kind in ("DD", "AD")}
    plan.close()
    g.close()
    return out if rank == 0 else None


def _cfg5_rank0(g, n, m, seed, var, reml_iters, out):
    """configs[4] on rank 0 (the drop-in API as one process): A and D GRMs, the 5-GRM REML and P / Py
    from its estimate; fills out["grm"], out["reml"], out["projection_s"]."""
    import ctypes
    from gmat_amd import dist
    from gmat_amd import _native as N
    from gmat_amd.uvlmm.uvlmm_varcom import _wemai_multi_gmat, projection
    from scipy.sparse import identity
    lib = N.ensure_device()
    with dist.local():
        mats, grm = [], {}
        for kind, name in ((0, "A"), (1, "D")):
            k = np.empty((n, n))
            sc = ctypes.c_double()
            t1 = time.perf_counter()
            N.check(lib.gmat_grm(g.handle, kind, 0.001, N.ptr(k), ctypes.byref(sc)), "gmat_grm")
            st = np.zeros(4)
            N.check(lib.gmat_grm_stats(N.ptr(st)), "gmat_grm_stats")
            grm[name] = {"kernel_ms": st[0] * 1e3, "wall_ms": (time.perf_counter() - t1) * 1e3,
                         "gflops_kernel": 2.0 * n * n * m / st[0] / 1e9,
                         "mx_frac_of_peak": st[1] / st[0] / 1e12 / MX_PEAK_TFLOPS,
                         "int8_equiv_frac_of_peak": st[1] / st[0] / 1e12 / INT8_PEAK_TOPS}
            mats.append(k)
        a, d = mats
        gl = [a, d, a * a, a * d, d * d]
        rng = np.random.Generator(np.random.PCG64(seed + 1))
        y = np.ones(n)
        for k, s_ in zip(gl, var[:5]):
            y += np.sqrt(s_) * (np.linalg.cholesky(k + 1e-3 * np.eye(n)) @ rng.standard_normal(n))
        y += np.sqrt(var[5]) * rng.standard_normal(n)
        t1 = time.perf_counter()
        est = _wemai_multi_gmat(y, np.ones((n, 1)), identity(n, format="csr"), gl, maxiter=reml_iters)
        st = np.zeros(4)
        N.check(lib.gmat_reml_stats(N.ptr(st)), "gmat_reml_stats")
        out["reml"] = {"iters": int(st[1]), "maxiter": reml_iters, "converged": bool(int(st[1]) < reml_iters),
                       "ms_per_iter": st[2] * 1e3, "wall_s": time.perf_counter() - t1,
                       "fp64_tflops": st[3] / st[2] / 1e12 if st[2] else None,
                       "frac": st[3] / st[2] / 1e12 / FP64_PEAK_TFLOPS if st[2] else None,
                       "var": [float(v) for v in est], "simulated": var.tolist(),
                       "scans_use": "the REML estimate (var)"}
        tr = getattr(_wemai_multi_gmat, "last_trace", None)
        if tr is not None and tr.size:
            out["reml"].update({"grad_norm_last5": tr[0, -5:].tolist(), "update_norm_last5": tr[1, -5:].tolist(),
                                "em_weight_last5": tr[2, -5:].tolist(), "grad_norm_min": float(tr[0].min()),
                                "update_norm_min": float(tr[1].min()),
                                "iters_with_em_weight": int(np.sum(tr[2] > 0))})
        out["grm"] = grm
        t1 = time.perf_counter()
        pvp, py = projection(y, np.ones((n, 1)), identity(n, format="csr"), gl, np.asarray(est, dtype=float))
        out["projection_s"] = time.perf_counter() - t1
    return pvp, py


def cfg5_main(args):
    """bench.py --config cfg5: the configs[4] leg alone, as its own JSON line."""
    from gmat_amd import dist
    backend = dist.init()
    rank, ws, _ = dist.world()
    rec = cfg5_leg(args.n_id, args.n_snp, args.p_cut, args.seed, args.reml_iters, rank, ws, backend,
                   family_size=args.family_size or None, reps=args.cfg5_reps)
    if rank == 0:
        out = {"metric": "SNP-pairs tested/sec (whole node), configs[4]", "value": rec["pairs_per_s"],
               "unit": "SNP-pairs/s", "n_gpus": ws, "higher_is_better": True, "data": "synthetic",
               "dtype": "fp6xfp4/fp64", "config": {"workload": rec["workload"], "n_id": args.n_id,
                                                   "n_snp": args.n_snp, "p_cut": args.p_cut,
                                                   "parallelism": rec["parallelism"]}}
        out.update({k: v for k, v in rec.items() if k not in ("workload", "parallelism")})
        print(json.dumps(out), flush=True)


def dry_run(args):
    """Every rank initialises the process group (the backend bench.py would use), the ranks
    all-reduce their rank numbers, and rank 0 prints one JSON line."""
    from gmat_amd import dist
    backend = dist.init()
    rank, ws, local = dist.world()
    total = dist.allreduce_sum(rank)
    mx = dist.allreduce_max(rank)
    dist.barrier()
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": ws, "backend": backend, "rank_sum": total, "rank_max": mx,
                          "launcher": os.environ.get("GMAT_LAUNCHER", "external" if ws > 1 else "none")}), flush=True)
    if total != ws * (ws - 1) / 2 or mx != ws - 1:
        sys.exit(4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n-id", type=int, default=2000)
    ap.add_argument("--n-snp", type=int, default=50000)
    ap.add_argument("--p-cut", type=float, default=1e-5)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-grm", action="store_true")
    ap.add_argument("--no-eff", action="store_true")
    ap.add_argument("--no-reml", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-cov", action="store_true")
    ap.add_argument("--no-split", action="store_true", help="skip the serial per-part rehearsal of the N-GPU split")
    ap.add_argument("--full-triangle", action="store_true",
                    help="recompute the exhaustive (unscreened) scan live for the full-triangle check (~2 min / N)")
    ap.add_argument("--config", default="cfg3", choices=["cfg3", "cfg5"],
                    help="cfg3: the headline (configs[2]/[3]); cfg5: configs[4] (5,000 x 100,000, 5 GRMs, epiDD/epiAD)")
    ap.add_argument("--reml-iters", type=int, default=200, help="configs[4] REML: maxiter (the reference's default)")
    ap.add_argument("--no-cfg5", action="store_true", help="skip the configs[4] leg of the default line")
    ap.add_argument("--family-size", type=int, default=0,
                    help="configs[4] cohort: full-sib family size of the last generation (0: random mating, the "
                         "SURVEY.md 8(d) generator)")
    ap.add_argument("--cfg5-reps", type=int, default=3, help="configs[4]: timed scans per kind (median reported)")
    ap.add_argument("--covariates", action="store_true",
                    help="profiling: the timed step uses the covariate design of the covariates leg")
    ap.add_argument("--allow-shared-gpu", action="store_true",
                    help="tests only: let --gpus N exceed the visible GPUs (ranks share devices, exchanges over gloo)")
    ap.add_argument("--hits-out", default=None, help="rank 0 writes the last step's merged hits to this .npz")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / process-group check only: every rank joins the group, exchanges its rank and "
                         "exits (no GPU work)")
    args = ap.parse_args()
    # --gpus N without a launcher: start N ranks of this script now, before anything in this process
    # touches the GPU (gmat_amd.launch), and exit with their status; a WORLD_SIZE that contradicts
    # --gpus is an error
    from gmat_amd import launch
    if args.allow_shared_gpu:
        os.environ["GMAT_ALLOW_SHARED_GPU"] = "1"  # inherited by the ranks
    rc = launch.main_or_spawn(args.gpus, os.path.abspath(__file__), sys.argv[1:], allow_shared=args.allow_shared_gpu)
    if rc is not None:
        sys.exit(rc)
    if args.dry_run:
        return dry_run(args)
    if args.config == "cfg5":
        if args.n_id == 2000:
            args.n_id = 5000
        if args.n_snp == 50000:
            args.n_snp = 100000
        return cfg5_main(args)

    from gmat_amd import dist
    from gmat_amd import _native as N
    backend = dist.init()
    rank, ws, _ = dist.world()
    N.ensure_device()
    # GPUs this job's ranks run on (one node, rank r on device LOCAL_RANK mod visible)
    devices_used = min(ws, N.device_count())
    n, m = args.n_id, args.n_snp
    var = np.array([0.4, 0.2, 0.4])
    geno, g, pvp, py, ka, y = build_inputs(n, m, args.seed, var, rank, ws, covariates=args.covariates)

    from gmat_amd.remma._scan import EpiPlan
    lib = N.ensure_device()
    lib.gmat_device_synchronize()
    # the first plan of a process also pays the solver libraries' first-use cost (code objects,
    # workspaces); the plan of the timed scan is the second one, as for every later remma call
    t_cold = time.perf_counter()
    if rank == 0:
        EpiPlan(g, pvp, py).close()
    t_cold = time.perf_counter() - t_cold
    dist.barrier()
    t_plan = time.perf_counter()
    plan = dist.shared_plan(g, pvp, py)  # spectral state computed on rank 0, imported by the others
    t_plan = time.perf_counter() - t_plan
    rows = dist.rank_rows("AA", m, rank, ws)
    total_pairs = m * (m - 1) // 2

    def step():
        return plan.scan("AA", rows, args.p_cut)

    t_first = time.perf_counter()
    for _ in range(args.warmup):
        step()
    t_first = time.perf_counter() - t_first
    setup = plan.setup_stats()
    setup["plan_create_wall_s"] = t_plan
    setup["first_plan_in_process_wall_s"] = t_cold
    setup["warmup_wall_s"] = t_first

    def sync():
        N.check(lib.gmat_device_synchronize(), "gmat_device_synchronize")

    dist.barrier()
    sync()
    t0 = time.perf_counter()
    screen_s = launches = ops = cands = hits = side_s = ref_s = 0.0
    ks, kx = {}, {}
    n_slice = 0
    for it in range(args.steps):
        res = step()
        if it == args.steps - 1:  # the candidate kernels' HIP-event times of the last step (reading them
            # every step was ~60 us of host time per step; they are scaled to the steps below)
            for name, v in plan.kernel_stats_ext().items():
                kx[name] = {key: v[key] * args.steps for key in ("s", "launches", "pairs")}
        st = plan.stats()
        screen_s += st["screen_s"]
        launches += st["launches"]
        ops += st["int8_ops"]
        cands += st["candidates"]
        side_s += st["side_s"]
        ref_s += st["refine_s"]
        n_slice = int(st["n_slice"])
        hits += res[0].size
        for k, v in plan.kernel_stats().items():
            ks[k] = ks.get(k, 0.0) + v
    sync()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    t_max = dist.allreduce_max(elapsed)
    hits_all = dist.allreduce_sum(hits) / args.steps
    cands_all = dist.allreduce_sum(cands) / args.steps

    # roofline of the dominant kernel (by kernel time per step): its MFMA ops per launch / its average
    # launch time, both from the library's own accounting (HIP events recorded on the kernel's own
    # stream, gmat_epi_kernel_stats).  prefilter_pass_kernel: 4 fp4 code products + 2 int8 E3 slices
    # over n_pad individuals per pair of every tile that runs = 16 n_pad fp4-equivalent ops per pair
    # (an int8 op counted twice: half the fp4 rate); lrc_screen_kernel: R x n_pad MACs x 2 per slot pair.
    from tools.pmc_summary import source_sha256
    kern_rec = {}
    for name, t_key, n_key, o_key, what in (
            ("prefilter_pass_kernel", "prefilter_s", "prefilter_launches", "prefilter_ops",
             "fp4-equivalent MFMA ops (fp4 + 2 x int8) of the tiles that run: 16 n_pad per pair "
             "(4 fp4 code products, 2 int8 E3 slices)"),
            ("lrc_screen_kernel", "screen_s", "screen_launches", "screen_ops",
             "fp6 x fp4 ops: R x n_pad MACs x 2 per slot pair (R = %d bottom eigen-directions of P, empty slot "
             "columns included)" % plan.lowrank_rank())):
        if ks.get(n_key, 0) > 0 and ks.get(t_key, 0) > 0:
            t_launch = ks[t_key] / ks[n_key]
            kern_rec[name] = {"kernel_s_per_step": ks[t_key] / args.steps, "avg_launch_ms": t_launch * 1e3,
                              "ops_per_launch": ks[o_key] / ks[n_key],
                              "achieved": ks[o_key] / ks[n_key] / t_launch / 1e12, "ops_note": what}
    # the candidate kernels (HIP events around each launch, gmat_epi_kernel_stats_ext), each against the
    # roof that binds it: pair_mxr_kernel issues n_pad^2 (1 + 1 / nK) fp6 x fp4 MACs x 2 per pair (the
    # block-upper P tiles), refine8_kernel R8_S = 7 int8 slices over the block-upper 32 x 64 tiles
    # (1,056 at n_pad 2,048) x 2 ops per pair; pair_side_kernel and refine8_side_kernel gather rows
    # (fp16 P x codes + int8 codes: 6 n_pad bytes per pair; fp64 P x codes + int8 codes: 20 n_pad)
    n_pad_k = -(-n // 256) * 256
    nK_k, NS_k, NB_k = n_pad_k // 128, n_pad_k // 64, n_pad_k // 32
    r8_tiles = NB_k * NS_k - ((NB_k // 2) * (NB_k // 2 - 1) if NB_k % 2 == 0 else (NB_k // 2) ** 2)
    for name, kname, per_pair, peak, unit, what in (
            ("pair_mx", "pair_mxr_kernel", 2.0 * 128 * 128 * nK_k * (nK_k + 1) / 2, MX_PEAK_TFLOPS, "TFLOP/s",
             "fp6 x fp4 ops of the block-upper P tiles per pair"),
            ("refine", "refine8_kernel", 2.0 * 7 * r8_tiles * 32 * 64, INT8_PEAK_TOPS, "TOP/s",
             "int8 ops: 7 slices of the block-upper 32 x 64 tiles per pair"),
            ("pair_side", "pair_side_kernel", 6.0 * n_pad_k, 8000.0, "GB/s", "gathered bytes per pair (HBM roof)"),
            ("refine_side", "refine8_side_kernel", 20.0 * n_pad_k, 8000.0, "GB/s", "gathered bytes per pair (HBM roof)")):
        v = kx.get(name)
        if not v or v["s"] <= 0:
            continue
        rate = v["pairs"] * per_pair / v["s"] / (1e12 if unit != "GB/s" else 1e9)
        kern_rec[kname] = {"kernel_s_per_step": v["s"] / args.steps, "launches_per_step": v["launches"] / args.steps,
                           "pairs_per_step": v["pairs"] / args.steps, "avg_launch_ms": v["s"] / v["launches"] * 1e3,
                           "achieved": rate, "unit": unit, "peak": peak, "frac": rate / peak, "ops_note": what,
                           "work_per_pair": per_pair,
                           "stats_source": "HIP events of the last timed step, scaled to the %d steps" % args.steps}
    screens = [k for k in ("prefilter_pass_kernel", "lrc_screen_kernel") if k in kern_rec]
    if screens:
        # the dominant kernel: the most work per step at its roof (issued ops / peak), not the longest
        # event span -- the candidate kernels' spans stretch while they share the CUs with the next
        # launch's prefilter, whose work per step is ~14x theirs
        dom = max(screens, key=lambda k: kern_rec[k]["ops_per_launch"] * kern_rec[k]["kernel_s_per_step"]
                  / kern_rec[k]["avg_launch_ms"])
        kr = kern_rec[dom]
        # fabric bytes per launch of this kernel from the PMC passes of tools/pmc.sh (FETCH_SIZE x 2 +
        # WRITE_SIZE); used only when recorded on the same kernel source (sha256 of the epi stage files), kernel,
        # rank and cohort size (else traffic stays null)
        def traffic_of(kname):
            tpath = os.path.join(REPO, "profiles", "traffic_%s.json" % kname)
            want = {"kernel": kname, "lowrank_rank": plan.lowrank_rank(), "n_id": n, "n_snp": m,
                    "source_sha256": source_sha256()}
            if not os.path.exists(tpath):
                return None, "no PMC record %s" % os.path.relpath(tpath, REPO)
            try:
                tj = json.load(open(tpath))
            except Exception as exc:
                return None, "unreadable: %s" % exc
            if all(tj.get(k) == v for k, v in want.items()):
                return tj.get("hbm_bytes_per_launch"), os.path.relpath(tpath, REPO)
            return None, "dropped: %s was recorded for %s" % (os.path.relpath(tpath, REPO), {k: tj.get(k) for k in want})

        traffic, traffic_src = traffic_of(dom)
        for kname, rec in kern_rec.items():
            rec["traffic_per_launch"], rec["traffic_source"] = traffic_of(kname)
        roofline = {"bound": "mfma", "achieved": kr["achieved"], "peak": MX_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": kr["achieved"] / MX_PEAK_TFLOPS, "traffic": traffic, "traffic_source": traffic_src,
                    "kernel": dom, "ops_note": kr["ops_note"], "avg_launch_ms": kr["avg_launch_ms"],
                    "issued_ops_per_launch": kr["ops_per_launch"], "kernels": kern_rec,
                    "fp64_equiv_tflops": total_pairs * (2.0 * n * n + 5 * n) / (t_max / args.steps) / 1e12}
        if dom == "prefilter_pass_kernel":
            # the prefilter's other roof: every tile streams its stage image per 64 individuals (+ its
            # test records) from L2 / MALL into LDS by LDS-DMA, and the chip moves ~6.4 TB/s of
            # LDS-DMA with every CU streaming (MI355X_MICROARCH.md, ldsdma-fill); the tile shape and
            # bytes are the plan's (gmat_epi_info)
            pi = plan.info()
            n_pad_ = pi["n_pad"]
            tiles_per_launch = kr["ops_per_launch"] / (16.0 * n_pad_) / (pi["pf_tile_rows"] * pi["pf_tile_cols"])
            dma_bytes = tiles_per_launch * (n_pad_ / 64 * pi["pf_stage_dma_bytes"] + pi["pf_tile_record_bytes"])
            dma_tbps = dma_bytes / (kr["avg_launch_ms"] * 1e-3) / 1e12
            roofline["lds_dma"] = {"bytes_per_launch": dma_bytes, "achieved_TBps": dma_tbps, "peak_TBps": LDS_DMA_PEAK_TBPS,
                                   "frac": dma_tbps / LDS_DMA_PEAK_TBPS, "tiles_per_launch": tiles_per_launch,
                                   "tile": [pi["pf_tile_rows"], pi["pf_tile_cols"]],
                                   "stage_bytes": pi["pf_stage_dma_bytes"], "record_bytes": pi["pf_tile_record_bytes"]}
    else:  # a level without per-kernel accounting (int8 / MX screens): the screen kernel's own stats
        avg_launch_s = screen_s / max(launches, 1)
        achieved = ops / max(launches, 1) / avg_launch_s / 1e12 if avg_launch_s > 0 else 0.0
        peak = MX_PEAK_TFLOPS if n_slice <= 0 else INT8_PEAK_TOPS
        roofline = {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
                    "traffic": None, "kernel": "screen level %d" % n_slice, "avg_launch_ms": avg_launch_s * 1e3,
                    "issued_ops_per_launch": ops / max(launches, 1)}

    # full-triangle check: the last step's hits merged over the ranks against the exhaustive scan
    merged = dist.gather_hits(res)
    live, t_live = None, None
    if args.full_triangle:
        ex_local, t_live = exhaustive_live(plan, rows, args.p_cut, lib)
        live = dist.gather_hits(ex_local)
        t_live = dist.allreduce_max(t_live)
    full_tri = full_triangle_check(g, pvp, py, merged, args.p_cut, live) if rank == 0 else None
    if rank == 0 and args.hits_out:
        np.savez(args.hits_out, i=merged[0], j=merged[1], eff=merged[2], var=merged[3], chi=merged[4], p=merged[5])
    if rank == 0 and t_live is not None:
        full_tri["exhaustive_s"] = t_live
        full_tri["exhaustive_pairs_per_s"] = total_pairs / t_live
    cpu = parity = None
    if rank == 0 and ws == 1 and not args.no_cpu:
        log("cpu baseline (oracle port) on stratified rows, %.0f s budget" % args.cpu_budget)
        cpu, used_rows, exp_hits = cpu_baseline(geno, pvp, py, args.cpu_budget)
        log("parity of the sampled rows against the oracle")
        parity = parity_check(plan, used_rows, exp_hits, args.p_cut)
    grm = reml = None
    if rank == 0 and not args.no_grm:
        with dist.local():
            log("configs[1] GRM")
            grm = grm_bench(n, 20000, args.seed)
            if not args.no_reml:
                log("configs[1] REML")
                reml = reml_bench(grm_bench.last_k, args.seed)
    split = None
    if rank == 0 and ws == 1 and not args.no_split:
        log("multi-GPU split rehearsed part by part")
        split = split_emulation(plan, m, args.p_cut, t_max / args.steps * 1e3, int(round(hits_all)), lib)
    cov = None
    if rank == 0 and ws == 1 and not args.no_cov:
        log("covariate design")
        cov = covariate_bench(g, ka, y, n, m, args.p_cut, args.seed, 2, t_max / args.steps * 1e3)
    e2e = None
    if rank == 0 and ws == 1 and not args.no_e2e:
        log("end to end remma_epiAA")
        e2e = e2e_bench(geno, ka, y, var, args.p_cut, int(round(hits_all)))
    eff = None
    if rank == 0 and ws == 1 and not args.no_eff:
        log("effect screen")
        eff = eff_bench(g, pvp, py, plan, n, m, args.p_cut, args.seed, geno=geno, cpu_budget=args.cpu_budget)
    plan.close()
    g.close()
    cfg5 = None
    if not args.no_cfg5:  # every rank: the configs[4] scans are sharded like configs[3]
        log("configs[4] leg")
        cfg5 = cfg5_leg(5000, 100000, args.p_cut, args.seed, args.reml_iters, rank, ws, backend,
                        family_size=args.family_size or None, reps=args.cfg5_reps)
    if rank == 0:
        if parity is None:
            parity = {}
        parity["full_triangle"] = full_tri
        value = total_pairs * args.steps / t_max
        out = {"metric": METRIC, "value": value, "unit": "SNP-pairs/s", "n_gpus": ws, "devices_used": devices_used,
               "backend": backend or "single", "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": t_max / args.steps * 1e3, "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "fp6xfp4/fp64" if n_slice <= 0 else "int8/fp64", "data": "synthetic",
               "config": {"workload": "configs[2]/[3]: exhaustive exact remma_epiAA, synthetic related cohort "
                                      "%d ind x %d SNP, p_cut=%g, %d pairs per step" % (n, m, args.p_cut, total_pairs),
                          "n_id": n, "n_snp": m, "p_cut": args.p_cut, "kind": "AA",
                          "parallelism": "rows folded over %d rank(s) (parallel=[N,k] split), backend %s"
                                         % (ws, backend or "single")},
               "roofline": roofline, "cpu_baseline": cpu, "parity": parity, "setup": setup, "grm": grm,
               "reml": reml, "end_to_end": e2e, "covariates": cov, "eff_screen": eff, "split_rehearsal": split,
               "cfg5": cfg5,
               "scan": {"hits_per_step": hits_all, "candidates_per_step": cands_all,
                        "screen_s_per_step_rank0": screen_s / args.steps, "side_s_per_step_rank0": side_s / args.steps,
                        "refine_s_per_step_rank0": ref_s / args.steps}}
        print(json.dumps(out), flush=True)
    if parity is not None and not parity.get("identical", True):
        log("PARITY FAILURE: GPU hits differ from the oracle on the sampled rows")
        sys.exit(3)
    if full_tri is not None and full_tri.get("checked") and not full_tri["identical"]:
        log("PARITY FAILURE: the step's hits differ from the exhaustive scan's")
        sys.exit(3)


if __name__ == "__main__":
    main()
