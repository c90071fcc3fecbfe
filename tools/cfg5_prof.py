"""Profiling driver for configs[4]'s scans: the 5,000 x 100,000 random-mating cohort of bench.py's cfg5
leg, P from the simulated variance components (no REML), one warm-up epiDD scan and one timed, so that
rocprofv3 --kernel-trace shows a configs[4] scan (tools/step_timeline.py on the trace).
    python tools/cfg5_prof.py [KIND]"""
import ctypes
import sys
import time

import numpy as np
from scipy.sparse import identity

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from gmat_amd import _native as N, synth  # noqa: E402
from gmat_amd.plink import Geno  # noqa: E402
from gmat_amd.remma._scan import EpiPlan  # noqa: E402
from gmat_amd.uvlmm.uvlmm_varcom import projection  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "DD"
    n, m = 5000, 100000
    lib = N.ensure_device()
    geno = synth.simulate_genotypes(n, m, seed=1)
    body = np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8)
    g = Geno(body=body, n_id=n, n_snp=m)
    mats = []
    for k_ in (0, 1):
        k = np.empty((n, n))
        sc = ctypes.c_double()
        N.check(lib.gmat_grm(g.handle, k_, 0.001, N.ptr(k), ctypes.byref(sc)), "gmat_grm")
        mats.append(k)
    a, d = mats
    gl = [a, d, a * a, a * d, d * d]
    var = np.array([0.3, 0.1, 0.1, 0.05, 0.05, 0.4])
    rng = np.random.default_rng(2)
    y = 1.0 + rng.standard_normal(n)
    pvp, py = projection(y, np.ones((n, 1)), identity(n, format="csr"), gl, var)
    plan = EpiPlan(g, pvp, py)
    rows = np.arange(m if kind == "AD" else m - 1, dtype=np.int64)
    for it in range(2):
        lib.gmat_device_synchronize()
        t0 = time.perf_counter()
        res = plan.scan(kind, rows, 1e-5)
        lib.gmat_device_synchronize()
        print("%s scan %d: %.3f s, %d hits, stats %s" % (kind, it, time.perf_counter() - t0, res[0].size, plan.stats()),
              flush=True)
    plan.close()
    g.close()


if __name__ == "__main__":
    main()
