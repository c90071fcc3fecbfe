"""Timing-only diagnostics of the low-rank screen (GMAT_LR_DIAG): full kernel, no stage loads, no
MFMAs, neither; screen seconds per full scan of one cohort (the diagnostic modes report no pairs).

    python tools/lr_diag.py --modes 0,1,2,3 --rounds 3 --n-snp 50000
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="0,1,2,3")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--n-id", type=int, default=2000)
    ap.add_argument("--n-snp", type=int, default=50000)
    ap.add_argument("--p-cut", type=float, default=1e-5)
    args = ap.parse_args()
    import bench
    from gmat_amd import _native as N
    from gmat_amd.remma._scan import EpiPlan
    N.ensure_device()
    geno, g, pvp, py = bench.build_inputs(args.n_id, args.n_snp, 1, np.array([0.4, 0.2, 0.4]), 0, 1)[:4]
    plan = EpiPlan(g, pvp, py)
    rows = np.arange(args.n_snp - 1)
    modes = [int(v) for v in args.modes.split(",")]
    res = {v: [] for v in modes}
    for r in range(args.rounds + 1):
        for v in modes:
            os.environ["GMAT_LR_DIAG"] = str(v)
            plan.scan("AA", rows, args.p_cut)
            st = plan.stats()
            if r:
                res[v].append(st["screen_s"])
    os.environ.pop("GMAT_LR_DIAG")
    for v in modes:
        t = np.array(res[v])
        print("diag %d: screen median %.4f s  min %.4f s" % (v, np.median(t), t.min()), flush=True)


if __name__ == "__main__":
    main()
