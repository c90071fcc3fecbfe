"""Full-triangle audit of the certified screens.

The screened scan (prefilter -> low-rank spectral screen -> pair screen -> exact fp64 refine) is
compared with the exhaustive scan (gmat_epi_scan level GMAT_SCREEN_NONE: every pair of the
triangle sent to the same fp64 refine kernel, the reference's computation remma_epiAA.py:71-82)
over the WHOLE pair set of a cohort, at several p_cut.  The refine of a pair does not depend on
the list it comes in, so the hit sets must be identical and their eff / var / chi / p
byte-identical.

    python tools/full_triangle.py [--n-id 2000 --n-snp 50000 --kind AA] --out DIR

Writes DIR/full_triangle_<kind>_<n>x<m>.json (the diff per p_cut, timings, how many pairs lie
within 2x of each threshold) and DIR/exhaustive_hits_<kind>_<n>x<m>.npz (the exhaustive hits at
the smallest p_cut: what bench.py compares each timed step against).
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def log(*a):
    print(*a, flush=True)


def cohort_fingerprint(g, pvp, py):
    """sha256 over the panel's per-SNP dosage sums and heterozygote counts, P and Py (guards a
    recorded exhaustive hit set; the same on every rank)."""
    h = hashlib.sha256()
    for a in (g.sum_dose, g.n_het, pvp, py):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def values_digest(hits):
    """sha256 of (i, j, eff, var, chi, p) bytes in (i, j) order."""
    h = hashlib.sha256()
    for a in hits:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def diff(scr, exh):
    """Symmetric difference of the (i, j) sets and byte equality of the common rows."""
    ks = set(zip(scr[0].tolist(), scr[1].tolist()))
    ke = set(zip(exh[0].tolist(), exh[1].tolist()))
    only_s, only_e = sorted(ks - ke), sorted(ke - ks)
    same_vals = False
    if not only_s and not only_e:
        same_vals = all(np.array_equal(np.asarray(a).view(np.uint64) if a.dtype == np.float64 else a,
                                       np.asarray(b).view(np.uint64) if b.dtype == np.float64 else b)
                        for a, b in zip(scr, exh))
    return {"screened_hits": len(ks), "exhaustive_hits": len(ke), "only_screened": len(only_s),
            "only_exhaustive": len(only_e), "symmetric_difference": len(only_s) + len(only_e),
            "values_byte_identical": bool(same_vals), "missed_examples": [list(map(int, t)) for t in only_e[:10]],
            "extra_examples": [list(map(int, t)) for t in only_s[:10]]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-id", type=int, default=2000)
    ap.add_argument("--n-snp", type=int, default=50000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--kind", default="AA", choices=["AA", "AD", "DD"])
    ap.add_argument("--p-cuts", default="1e-5,1e-4,1e-3")
    ap.add_argument("--pairs-per-call", type=float, default=6e7, help="exhaustive rows per call (progress lines)")
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "full_triangle"))
    ap.add_argument("--audit-pairs", type=int, default=200000)
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    import bench
    from gmat_amd import _native as N
    from gmat_amd.remma._scan import EpiPlan
    lib = N.ensure_device()
    n, m, kind = args.n_id, args.n_snp, args.kind
    p_cuts = sorted(float(x) for x in args.p_cuts.split(","))
    t0 = time.time()
    geno, g, pvp, py, ka, y = bench.build_inputs(n, m, args.seed, np.array([0.4, 0.2, 0.4]), 0, 1)
    log("cohort %d x %d ready in %.1f s" % (n, m, time.time() - t0))
    fp = cohort_fingerprint(g, pvp, py)
    plan = EpiPlan(g, pvp, py)
    rows = np.arange(m if kind == "AD" else m - 1, dtype=np.int64)
    total = float(m) * m if kind == "AD" else m * (m - 1) / 2.0
    rec = {"config": {"n_id": n, "n_snp": m, "seed": args.seed, "kind": kind, "pairs": total,
                      "cohort": "bench.py build_inputs (related synthetic cohort, [A, AxA] REML-free P at (0.4, 0.2, 0.4))",
                      "fingerprint_sha256": fp},
           "lowrank_rank": plan.lowrank_rank(), "screened": {}, "exhaustive": {}, "diff": {}}
    screened = {}
    for pc in p_cuts:
        for ns, name in ((0, "auto"), (-1, "mx")):
            if name == "mx" and pc != p_cuts[0]:
                continue
            t1 = time.perf_counter()
            res = plan.scan(kind, rows, pc, n_slice=ns)
            lib.gmat_device_synchronize()
            dt = time.perf_counter() - t1
            st = plan.stats()
            screened[(pc, name)] = res
            rec["screened"]["%g/%s" % (pc, name)] = {"s": dt, "hits": int(res[0].size), "candidates": st["candidates"],
                                                    "screen_level": int(st["n_slice"])}
            log("screened %s p_cut %g: %d hits, %.0f candidates, %.2f s" % (name, pc, res[0].size, st["candidates"], dt))
    # exhaustive at the largest p_cut, rows in calls of about pairs_per_call pairs (progress lines)
    pmax = p_cuts[-1]
    per_row = (np.full(rows.size, m, dtype=np.float64) if kind == "AD" else (m - 1 - rows).astype(np.float64))
    cum = np.cumsum(per_row)
    parts, done, t_ex, r0 = [], 0.0, 0.0, 0
    near = {pc: 0 for pc in p_cuts}
    while r0 < rows.size:
        r1 = int(np.searchsorted(cum, (cum[r0 - 1] if r0 else 0.0) + args.pairs_per_call, side="right"))
        r1 = max(r1, r0 + 1)
        t1 = time.perf_counter()
        res = plan.scan(kind, rows[r0:r1], max(pmax * 2, pmax), n_slice=N.GMAT_SCREEN_NONE)
        t_ex += time.perf_counter() - t1
        done += float(per_row[r0:r1].sum())
        for pc in p_cuts:  # pairs just above each threshold (the screens had to reject them)
            near[pc] += int(np.sum((res[5] >= pc) & (res[5] < 2 * pc)))
        keep = res[5] < pmax
        parts.append(tuple(a[keep] for a in res))
        log("exhaustive rows [%d, %d): %.3g / %.3g pairs, %.1f s, %.3g pairs/s" % (r0, r1, done, total, t_ex, done / t_ex))
        r0 = r1
    exh = tuple(np.concatenate([p[t] for p in parts]) for t in range(6))
    rec["exhaustive"] = {"s": t_ex, "pairs_per_s": total / t_ex, "hits_at_max_p_cut": int(exh[0].size),
                         "fp64_tflops": total * (2.0 * n * n + 5 * n) / t_ex / 1e12}
    ok = True
    for pc in p_cuts:
        sel = exh[5] < pc
        e_pc = tuple(a[sel] for a in exh)
        for name in ("auto", "mx"):
            if (pc, name) not in screened:
                continue
            d = diff(screened[(pc, name)], e_pc)
            d["pairs_within_2x_above_p_cut"] = near[pc]
            rec["diff"]["%g/%s" % (pc, name)] = d
            ok = ok and d["symmetric_difference"] == 0 and d["values_byte_identical"]
            log("p_cut %g %s: %s" % (pc, name, json.dumps(d)))
    rec["identical"] = bool(ok)
    # certificate audit: exact var / certified lower bound over random pairs of the triangle and the
    # pairs just above the smallest threshold (the ones the screens must reject with least room)
    rng = np.random.default_rng(7)
    ri = rng.integers(0, m - 1, 600000)
    rj = rng.integers(0, m, 600000)
    keep = (ri < rj) if kind != "AD" else np.ones(ri.size, bool)
    samp = np.column_stack([ri[keep], rj[keep]])[:args.audit_pairs]
    near_pairs = np.column_stack([exh[0], exh[1]])[(exh[5] >= p_cuts[0]) & (exh[5] < 2 * p_cuts[0])]
    rec["audit"] = {}
    for name, pr in (("random", samp), ("near_threshold", near_pairs)):
        if not pr.shape[0]:
            continue
        t1 = time.perf_counter()
        _, var, _, _ = plan.pairs(kind, pr)
        lb = plan.audit(kind, pr)
        a = {"pairs": int(pr.shape[0]), "s": time.perf_counter() - t1}
        for col, scr in ((0, "prefilter"), (1, "lowrank")):
            pos = lb[:, col] > 0
            r = var[pos] / lb[pos, col]
            a[scr] = {"bound_positive": int(pos.sum()), "min_ratio_var_over_bound": float(r.min()) if r.size else None,
                      "median_ratio": float(np.median(r)) if r.size else None}
            ok = ok and (not r.size or float(r.min()) >= 1.0)
        rec["audit"][name] = a
        log("audit %s: %s" % (name, json.dumps(a)))
    rec["identical"] = bool(ok)
    p0 = p_cuts[0]
    sel = exh[5] < p0
    h0 = tuple(a[sel] for a in exh)
    rec["exhaustive_hits_sha256_at_%g" % p0] = values_digest(h0)
    tag = "%s_%dx%d" % (kind, n, m)
    np.savez_compressed(os.path.join(args.out, "exhaustive_hits_%s.npz" % tag), i=h0[0].astype(np.int32),
                        j=h0[1].astype(np.int32), eff=h0[2], var=h0[3], chi=h0[4], p=h0[5], p_cut=np.array([p0]),
                        fingerprint=np.frombuffer(bytes.fromhex(fp), dtype=np.uint8))
    with open(os.path.join(args.out, "full_triangle_%s.json" % tag), "w") as f:
        json.dump(rec, f, indent=1)
    log(json.dumps({"identical": rec["identical"], "exhaustive_s": t_ex, "hits": int(h0[0].size)}))
    plan.close()
    g.close()
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())
