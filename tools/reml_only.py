"""Profiling driver: only the configs[1] REML -- 2-GRM ([A, AxA]) weighted EM-AI REML at n = 2,000
on a synthetic related cohort (bench.py's reml leg without the scan), so rocprofv3 sees its kernels."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from gmat_amd import _native as N, synth  # noqa: E402
from gmat_amd.plink import Geno  # noqa: E402
from gmat_amd.uvlmm.uvlmm_varcom import _wemai_multi_gmat  # noqa: E402
from scipy.sparse import identity  # noqa: E402

n, m = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (2000, 20000)))
lib = N.ensure_device()
geno = synth.simulate_genotypes(n, m, seed=12)
g = Geno(body=np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8), n_id=n, n_snp=m)
k = np.empty((n, n))
sc = ctypes.c_double()
N.check(lib.gmat_grm(g.handle, 0, 0.001, N.ptr(k), ctypes.byref(sc)), "gmat_grm")
g.close()
rng = np.random.Generator(np.random.PCG64(4))
kk = k * k
y = np.ones(n)
for gm, s_ in ((k, 0.4), (kk, 0.2)):
    y += np.sqrt(s_) * (np.linalg.cholesky(gm + 1e-4 * np.eye(n)) @ rng.standard_normal(n))
y += np.sqrt(0.4) * rng.standard_normal(n)
for rep in range(2):
    t0 = time.perf_counter()
    var = _wemai_multi_gmat(y, np.ones((n, 1)), identity(n, format="csr"), [k, kk])
    st = np.zeros(4)
    N.check(lib.gmat_reml_stats(N.ptr(st)), "gmat_reml_stats")
    print("REML %d iterations, %.2f ms/iter (%.2f TF/s), wall %.3f s, var %s" % (
        st[1], st[2] * 1e3, st[3] / st[2] / 1e12, time.perf_counter() - t0, np.round(var, 4)), flush=True)
