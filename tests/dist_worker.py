"""Worker for tests/test_dist_cpu.py: one rank of a gloo (CPU) run of the sharded scan.

The per-rank compute is the CPU oracle here (test infrastructure); the sharding, the
genotype all-gather, the P broadcast and the hit merge are the product code in
gmat_amd/dist.py.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from gmat_amd import dist  # noqa: E402
from gmat_amd.plink import read_bed_body  # noqa: E402
from oracle import gmat_oracle as O  # noqa: E402


def main():
    out_path = sys.argv[1]
    dist.init("gloo")
    rank, ws, _ = dist.world()
    tiny = os.path.join(REPO, "tests", "golden", "tiny", "tiny")
    body, n, m = read_bed_body(tiny)
    nb = (n + 3) // 4
    lo, hi = dist.snp_shard(m, rank, ws)
    full = dist.allgather_packed(body.reshape(m, nb)[lo:hi], m, nb)
    assert np.array_equal(full, body), "all-gather mismatch"
    snp = O.read_plink(tiny)
    ref = np.load(os.path.join(REPO, "tests", "golden", "tiny", "tiny_ref.npz"))
    pvp = py = None
    if rank == 0:
        y, x, col, nid = O.design_matrix(tiny + ".pheno", tiny)
        a = ref["agmat"]
        pvp, py = O.projection(y, x, col, nid, [a, a * a], ref["var"])
        py = py[:, 0]
    pvp = dist.broadcast_array(pvp, 0, shape=(n, n))
    py = dist.broadcast_array(py, 0, shape=(n,))

    def scan_fn(kind, rows, p_cut):
        h = O.epi_scan(kind, snp, pvp, py.reshape(-1, 1), snp_lst_0=[int(r) for r in rows], p_cut=p_cut)
        i, j = h[:, 0].astype(np.int64), h[:, 1].astype(np.int64)
        with np.errstate(divide="ignore", invalid="ignore"):
            var = h[:, 2] ** 2 / h[:, 3]
        return i, j, h[:, 2], var, h[:, 3], h[:, 4]

    results = {}
    for kind in ("AA", "AD", "DD"):
        merged = dist.distributed_scan(scan_fn, kind, m, 0.05)
        if rank == 0:
            results[kind] = merged
    # shared_plan: rank 0's plan state reaches every rank byte for byte (plan stubbed: no GPU here)
    from gmat_amd.remma import _scan

    class StubPlan:
        def __init__(self, geno, pvp_, py_, state=None):
            self.state = state

        def export_state(self):
            return (np.arange(100003, dtype=np.int64) * 7919 % 251).astype(np.uint8)

    real = _scan.EpiPlan
    _scan.EpiPlan = StubPlan
    try:
        plan = dist.shared_plan(None, pvp, py)
    finally:
        _scan.EpiPlan = real
    want = StubPlan(None, None, None).export_state()
    state_ok = float(plan.state is None) if rank == 0 else float(np.array_equal(plan.state, want))
    state_ok = -dist.allreduce_max(-state_ok)  # min over ranks
    mx = dist.allreduce_max(float(rank))
    if rank == 0:
        np.savez(out_path, mx=mx, state_ok=state_ok, **{k + "_" + str(t): v[t] for k, v in results.items() for t in range(6)})
    dist.barrier()


if __name__ == "__main__":
    main()
