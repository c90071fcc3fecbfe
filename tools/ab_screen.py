"""In-process interleaved A/B of screen-kernel variants (GMAT_SCREEN_VARIANT) on one cohort.

    python tools/ab_screen.py --variants 0,1,2,3 --rounds 5 --n-snp 12000
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--n-id", type=int, default=2000)
    ap.add_argument("--n-snp", type=int, default=12000)
    ap.add_argument("--p-cut", type=float, default=1e-5)
    ap.add_argument("--env", default="GMAT_SCREEN_VARIANT", help="variant selector (GMAT_MX_VARIANT for the MX screen)")
    args = ap.parse_args()
    import bench
    from gmat_amd import _native as N
    from gmat_amd.remma._scan import EpiPlan
    N.ensure_device()
    geno, g, pvp, py = bench.build_inputs(args.n_id, args.n_snp, 1, np.array([0.4, 0.2, 0.4]), 0, 1)[:4]
    plan = EpiPlan(g, pvp, py)
    rows = np.arange(args.n_snp - 1)
    variants = [int(v) for v in args.variants.split(",")]
    res = {v: [] for v in variants}
    ref = None
    for r in range(args.rounds + 1):
        for v in variants:
            os.environ[args.env] = str(v)
            out = plan.scan("AA", rows, args.p_cut)
            st = plan.stats()
            if ref is None:
                ref = out
            else:
                assert all(np.array_equal(a, b) for a, b in zip(ref, out)), "variant %d changed the hits" % v
            if r:
                res[v].append(st["screen_s"])
    pairs = args.n_snp * (args.n_snp - 1) / 2
    for v in variants:
        t = np.array(res[v])
        print("variant %d: screen median %.4f s  min %.4f s  (%.1f M pairs/s screen-only)"
              % (v, np.median(t), t.min(), pairs / np.median(t) / 1e6))


if __name__ == "__main__":
    main()
