"""Profiling driver: bench.py's end-to-end leg alone (remma_epiAA from .bed/.bim/.fam/pheno files to the
hits file, configs[2] cohort), REPS calls, with the per-phase times of each call (remma._scan.LAST_PHASES).
Under rocprofv3 --kernel-trace --runtime-trace the last call shows where a call's time goes.
    python tools/e2e_only.py [REPS]"""
import json
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    n, m = 2000, 50000
    geno, g, pvp, py, ka, y = bench.build_inputs(n, m, 1, np.array([0.4, 0.2, 0.4]), 0, 1)
    g.close()
    r = bench.e2e_bench(geno, ka, y, np.array([0.4, 0.2, 0.4]), 1e-5, 10932, reps=reps)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
