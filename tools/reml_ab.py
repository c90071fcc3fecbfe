"""Device REML / SPD-inverse timing of one library build (GMAT_HIP_LIB selects it), for A/Bs of the f64
kernels (chol.hip, dgemm.hip): the configs[1] shape (2 GRMs, n = 2,000) and the configs[4] shape
(5 GRMs, n = 5,000, fixed iteration count), random SPD relationship matrices.
   GMAT_HIP_LIB=ab/lib_x.so python tools/reml_ab.py NAME"""
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def grm(rng, n, m):
    x = rng.standard_normal((n, m))
    return x @ x.T / m + 1e-2 * np.eye(n)


def main():
    from scipy.sparse import identity
    from gmat_amd import _native as N
    from gmat_amd.gmatrix import spd_inverse
    from gmat_amd.uvlmm.uvlmm_varcom import _wemai_multi_gmat
    lib = N.ensure_device()
    rng = np.random.default_rng(5)
    out = {"name": sys.argv[1], "lib": os.environ.get("GMAT_HIP_LIB", "gmat_amd/libgmat_hip.so")}
    for n, ng, iters in ((2000, 2, 30), (5000, 5, 20)):
        ks = [grm(rng, n, 1500) for _ in range(ng)]
        ks = [k if i % 2 == 0 else k * ks[0] for i, k in enumerate(ks)]
        y = 1.0 + rng.standard_normal(n)
        _wemai_multi_gmat(y, np.ones((n, 1)), identity(n, format="csr"), ks, maxiter=3)
        var = _wemai_multi_gmat(y, np.ones((n, 1)), identity(n, format="csr"), ks, maxiter=iters, cc_par=-1.0,
                                cc_gra=-1.0)
        st = np.zeros(4)
        N.check(lib.gmat_reml_stats(N.ptr(st)), "gmat_reml_stats")
        a = ks[0] + n * 1e-3 * np.eye(n)
        spd_inverse(a)
        t = []
        for _ in range(5):
            t0 = time.perf_counter()
            ai = spd_inverse(a)
            t.append(time.perf_counter() - t0)
        err = float(np.abs(ai @ a - np.eye(n)).max())
        out["n%d_g%d" % (n, ng)] = {"iters": int(st[1]), "ms_per_iter": st[2] * 1e3,
                                     "fp64_tflops": st[3] / st[2] / 1e12, "spd_inverse_ms": 1e3 * min(t),
                                     "inverse_residual": err,
                                     "sha": hashlib.sha256(ai.tobytes() + np.asarray(var).tobytes()).hexdigest()[:12]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
