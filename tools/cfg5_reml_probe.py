"""Probe: does the configs[4] 5-GRM REML ([A, D, AxA, AxD, DxD] + residual, uvlmm_varcom.py:41-99)
converge on bench.py's cfg5 cohort, and after how many iterations?  For each simulated variance
vector: iterations, convergence, the estimate, and the gradient / update norms and EM weights along
the way (gmat_reml_trace).
    python tools/cfg5_reml_probe.py FAMILY_SIZE MAXITER "0.3,0.1,0.1,0.05,0.05,0.4[@SEEDS]" ["..."]
SEEDS (e.g. "2-17"): phenotype draws (the bench's is seed + 1 = 2), one REML each."""
import ctypes
import json
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from gmat_amd import _native as N, synth  # noqa: E402
from gmat_amd.plink import Geno  # noqa: E402
from gmat_amd.uvlmm.uvlmm_varcom import _wemai_multi_gmat  # noqa: E402
from scipy.sparse import identity  # noqa: E402

fam = int(sys.argv[1]) or None
maxiter = int(sys.argv[2])
n, m, seed = 5000, 100000, 1
lib = N.ensure_device()
t0 = time.time()
geno, _ = synth.simulate_genotype_shard(n, m, 0, m, seed=seed, family_size=fam)
g = Geno(body=np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8), n_id=n, n_snp=m)
del geno
mats = []
for kind in (0, 1):
    k = np.empty((n, n))
    N.check(lib.gmat_grm(g.handle, kind, 0.001, N.ptr(k), ctypes.byref(ctypes.c_double())), "gmat_grm")
    mats.append(k)
g.close()
a, d = mats
gl = [a, d, a * a, a * d, d * d]
print("cohort + GRMs %.1f s" % (time.time() - t0), flush=True)
chol = [np.linalg.cholesky(k + 1e-3 * np.eye(n)) for k in gl]
print("factors %.1f s" % (time.time() - t0), flush=True)
runs = []
for spec in sys.argv[3:]:
    vs, _, seeds = spec.partition("@")
    lo_hi = [int(v) for v in (seeds or str(seed + 1)).split("-")]
    for ps in range(lo_hi[0], lo_hi[-1] + 1):
        runs.append((np.array([float(v) for v in vs.split(",")]), ps))
for var, ps in runs:
    rng = np.random.Generator(np.random.PCG64(ps))
    y = np.ones(n)
    for L, s_ in zip(chol, var[:5]):
        y += np.sqrt(s_) * (L @ rng.standard_normal(n))
    y += np.sqrt(var[5]) * rng.standard_normal(n)
    t1 = time.perf_counter()
    est = _wemai_multi_gmat(y, np.ones((n, 1)), identity(n, format="csr"), gl, maxiter=maxiter)
    tr = _wemai_multi_gmat.last_trace
    it = tr.shape[1]
    marks = [k for k in (1, 10, 50, 100, 200, 500, 1000, 2000, 5000) if k <= it] + [it]
    print(json.dumps({"family_size": fam, "pheno_seed": ps, "simulated": var.tolist(), "iters": it, "converged": it < maxiter,
                      "wall_s": time.perf_counter() - t1, "var": np.round(est, 5).tolist(),
                      "grad_norm_at": {k: float(tr[0, k - 1]) for k in marks},
                      "update_norm_at": {k: float(tr[1, k - 1]) for k in marks},
                      "iters_with_em_weight": int(np.sum(tr[2] > 0)),
                      "last_zero_weight_iter": int(np.max(np.nonzero(tr[2] == 0)[0]) + 1) if np.any(tr[2] == 0) else 0}),
          flush=True)
