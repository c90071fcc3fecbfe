"""Profiling driver for the multi-GPU split: the configs[2] cohort's part K of the N-way folded split
(dist.rank_rows, what rank K of an N-GPU run scans), scanned REPS times on this GPU, so that
rocprofv3 --kernel-trace shows one rank's step (tools/step_timeline.py on the trace).
    python tools/split_part.py [K N REPS]"""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import bench  # noqa: E402
from gmat_amd import _native as N, dist  # noqa: E402
from gmat_amd.remma._scan import EpiPlan  # noqa: E402


def main():
    k, ways, reps = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (0, 8, 5)))
    lib = N.ensure_device()
    n, m = 2000, 50000
    geno, g, pvp, py, ka, y = bench.build_inputs(n, m, 1, np.array([0.4, 0.2, 0.4]), 0, 1)
    plan = EpiPlan(g, pvp, py)
    rows = dist.rank_rows("AA", m, k, ways)
    plan.scan("AA", rows, 1e-5)
    for _ in range(reps):
        lib.gmat_device_synchronize()
        t0 = time.perf_counter()
        res = plan.scan("AA", rows, 1e-5)
        lib.gmat_device_synchronize()
        print("part %d of %d: %d rows, %.3f ms, %d hits, launches %d" % (
            k, ways, rows.size, (time.perf_counter() - t0) * 1e3, res[0].size, plan.stats()["launches"]), flush=True)
    plan.close()
    g.close()


if __name__ == "__main__":
    main()
