"""Profiling driver: only the configs[1] GRM (agmat kernels) -- a few gmat_grm calls on a
2,000 x 20,000 synthetic panel, so rocprofv3 PMC passes see nothing else."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from gmat_amd import _native as N, synth  # noqa: E402
from gmat_amd.plink import Geno  # noqa: E402

n, m = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (2000, 20000)))
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
lib = N.ensure_device()
geno = synth.simulate_genotypes(n, m, seed=12)
g = Geno(body=np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8), n_id=n, n_snp=m)
k = np.empty((n, n))
sc = ctypes.c_double()
st = np.zeros(4)
for kind in (0, 1):
    for _ in range(reps):
        N.check(lib.gmat_grm(g.handle, kind, 0.001, N.ptr(k), ctypes.byref(sc)), "gmat_grm")
        N.check(lib.gmat_grm_stats(N.ptr(st)), "gmat_grm_stats")
        print("kind %d: syrk %.1f us (%.3g TOP/s), all kernels %.1f us" % (kind, st[0] * 1e6, st[1] / st[0] / 1e12,
                                                                          st[3] * 1e6), flush=True)
g.close()
