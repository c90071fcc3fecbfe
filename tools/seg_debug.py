"""Debug driver of the segmented plans (epi_seg.hip): a small cohort scanned as one plan and in
segments, step by step with progress lines (run with GMAT_DEBUG=1 AMD_SERIALIZE_KERNEL=3)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from gmat_amd import synth
    from gmat_amd.plink import Geno
    from gmat_amd.remma._scan import EpiPlan
    from oracle import gmat_oracle as O
    n, m, seg = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    geno = synth.simulate_genotypes(n, m, seed=71)
    snp = np.ascontiguousarray(geno.T, dtype=np.float64)
    ka = O.agmat(snp[:, :3000])
    y = 1.0 + np.random.default_rng(71).standard_normal(n)
    pvp, py = O.projection(y, np.ones((n, 1)), np.arange(n), n, [ka, ka * ka], np.array([0.4, 0.2, 0.4]))
    py = py[:, 0]
    body = np.frombuffer(synth.pack_bed(geno)[3:], dtype=np.uint8)
    kinds = sys.argv[4].split(",") if len(sys.argv) > 4 else ["AA"]
    with Geno(body=body, n_id=n, n_snp=m) as g:
        ref = {}
        with EpiPlan(g, pvp, py) as plan:
            for kind in kinds:
                rows = np.arange(m - 1 if kind != "AD" else m, dtype=np.int64)
                ref[kind] = plan.scan(kind, rows, 1e-4)
                print("one plan", kind, ref[kind][0].size, flush=True)
        os.environ["GMAT_SEG_SNPS"] = seg
        with EpiPlan(g, pvp, py) as plan:
            print("segmented plan", plan.layout(), flush=True)
            for kind in kinds:
                rows = np.arange(m - 1 if kind != "AD" else m, dtype=np.int64)
                t0 = time.time()
                got = plan.scan(kind, rows, 1e-4)
                same = all(np.array_equal(np.asarray(u).view(np.uint64), np.asarray(v).view(np.uint64))
                           for u, v in zip(got, ref[kind]))
                print("segmented", kind, got[0].size, "identical", same, "%.2f s" % (time.time() - t0), flush=True)


if __name__ == "__main__":
    main()
