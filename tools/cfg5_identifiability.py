"""Why the configs[4] 5-GRM REML cannot meet the reference's stopping rule: the expected (average)
information of [A, D, AxA, AxD, DxD] + residual at the simulated variances, on bench.py's cohort
generator (gmat_amd/synth.py), CPU only.

For each cohort design it prints the information matrix's condition number, the asymptotic standard
error of each variance over its simulated value (sqrt(diag(I^-1)) / var) and the correlations of the
kernels' off-diagonal entries.  Kernels as bench.py builds them (A, D from centred dosages /
heterozygote indicators, the products elementwise, + 1e-3 I); I_kl = 1/2 tr(P K_k P K_l)
(uvlmm_varcom.py:64-75's AI at its expectation).

    python tools/cfg5_identifiability.py N_ID N_SNP
"""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from gmat_amd import synth  # noqa: E402


def kernels(geno):
    g = geno.T.astype(np.float64)  # n x m
    n = g.shape[0]
    p = g.mean(0) / 2
    x = g - 2 * p
    a = x @ x.T / np.sum(2 * p * (1 - p))
    h = (g == 1).astype(np.float64) - 2 * p * (1 - p)
    d = h @ h.T / np.sum((2 * p * (1 - p)) ** 2)
    a += 1e-3 * np.eye(n)
    d += 1e-3 * np.eye(n)
    return [a, d, a * a, a * d, d * d]


def information(ks, var):
    n = ks[0].shape[0]
    v = sum(s * k for s, k in zip(var, ks)) + var[-1] * np.eye(n)
    vi = np.linalg.inv(v)
    vx = vi @ np.ones((n, 1))
    p = vi - vx @ vx.T / vx.sum()
    pk = [p @ k for k in ks + [np.eye(n)]]
    c = len(pk)
    info = np.empty((c, c))
    for a in range(c):
        for b in range(a, c):
            info[a, b] = info[b, a] = 0.5 * np.sum(pk[a] * pk[b].T)
    return info


def report(name, geno, var):
    ks = kernels(geno)
    info = information(ks, var)
    se = np.sqrt(np.diag(np.linalg.inv(info)))
    ev = np.linalg.eigvalsh(info)
    off = np.corrcoef([k[np.triu_indices(k.shape[0], 1)] for k in ks])
    print("%s: cond %.3g  se/var %s  kernel correlations (A-D A-AA A-AD A-DD D-AA D-AD D-DD AA-AD AA-DD AD-DD) %s"
          % (name, ev[-1] / ev[0], np.round(se / np.asarray(var), 2), np.round(off[np.triu_indices(5, 1)], 2)),
          flush=True)


def main():
    n, m = int(sys.argv[1]), int(sys.argv[2])
    var = [0.3, 0.1, 0.1, 0.05, 0.05, 0.4]  # bench.py cfg5_leg
    t = time.time()
    report("random mating", synth.simulate_genotypes(n, m, seed=3), var)
    for f in (5, 20):
        report("full-sib families of %d" % f, synth.simulate_genotypes(n, m, seed=3, family_size=f), var)
    print("%.1f s" % (time.time() - t))


if __name__ == "__main__":
    main()
