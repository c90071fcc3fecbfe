"""Summarise tools/pmc.sh output: per-kernel counter totals and derived ratios.

    python tools/pmc_summary.py DIR KERNEL [--out traffic.json --level L --rank R --n-id N --n-snp M]

With --out, writes the traffic record bench.py uses for roofline.traffic: fabric bytes per launch
(FETCH_SIZE x 2, the gfx950 wide-read correction of MI355X_MICROARCH.md "HBM", + WRITE_SIZE), keyed
by the kernel, its screen level and low-rank rank, the cohort size and the sha256 of the epi stage files (the
kernels' source), so that a record of other code or another kernel shape is not used (bench.py
drops it).  Launch times under --pmc are those of serialised kernels (the profiler serialises
dispatches), so they are recorded but not compared.
"""
import argparse
import collections
import csv
import glob
import hashlib
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


EPI_SOURCES = ("epi.h", "epi_prefilter.hip", "epi_screen.hip", "epi_refine.hip", "epi_setup.hip", "epi_plan.hip",
               "epi_scan.hip")


def source_sha256(paths=None):
    """Fingerprint of the scan kernels' source (the epi.h / epi_*.hip stage files, in a fixed order): a
    traffic record applies only to the code it measured."""
    h = hashlib.sha256()
    for name in (EPI_SOURCES if paths is None else paths):
        with open(os.path.join(REPO, "gmat_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("kernel")
    ap.add_argument("--out")
    ap.add_argument("--level", type=int, default=-1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--n-id", type=int, default=0)
    ap.add_argument("--n-snp", type=int, default=0)
    args = ap.parse_args()
    d, key = args.dir, args.kernel
    agg = collections.defaultdict(float)
    dur = 0.0
    launches = 0
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if key in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    for f in sorted(glob.glob(os.path.join(d, "p1", "run_kernel_trace.csv"))):
        for r in csv.DictReader(open(f)):
            if key in r["Kernel_Name"]:
                dur += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
                launches += 1
    lines = ["kernel %s: %d launches, %.4f s, %.1f us per launch" % (key, launches, dur, dur / max(launches, 1) * 1e6)]
    lines.append(str({k: "%.4g" % v for k, v in sorted(agg.items())}))
    g = agg.get("GRBM_GUI_ACTIVE", 0) / 8
    if g:
        lines.append("clock GHz %.3f (GRBM_GUI_ACTIVE / 8 / kernel time)" % (g / dur / 1e9 if dur else 0))
        lines.append("MFMA busy (per SIMD) %.3f" % (agg["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / g))
    w = agg.get("SQ_WAVE_CYCLES", 0)
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            lines.append("%s / WAVE_CYCLES %.3f" % (k, agg[k] / w))
    m = agg.get("SQ_INSTS_MFMA", 0)
    if m:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"):
            if k in agg:
                lines.append("%s per MFMA %.2f" % (k, agg[k] / m))
    if "TCC_HIT_sum" in agg:
        lines.append("L2 hit %.3f" % (agg["TCC_HIT_sum"] / max(agg["TCC_HIT_sum"] + agg["TCC_MISS_sum"], 1)))
    if "FETCH_SIZE" in agg:
        lines.append("FETCH_SIZE (KB, x2 gfx950 correction) %.4g -> %.4g GB" % (agg["FETCH_SIZE"], 2 * agg["FETCH_SIZE"] * 1024 / 1e9))
    print("\n".join(lines))

    if args.out and "FETCH_SIZE" in agg:
        fetch = 2 * agg["FETCH_SIZE"] * 1024  # KB, gfx950 wide-read correction (MI355X_MICROARCH.md:298)
        write = agg.get("WRITE_SIZE", 0.0) * 1024
        rec = {"kernel": key, "screen_level": args.level, "lowrank_rank": args.rank, "n_id": args.n_id,
               "n_snp": args.n_snp, "source_sha256": source_sha256(), "launches": launches, "kernel_s": dur,
               "avg_launch_us": dur / max(launches, 1) * 1e6, "fetch_bytes": fetch, "write_bytes": write,
               "hbm_bytes_per_launch": (fetch + write) / max(launches, 1),
               "source": os.path.relpath(d), "summary": lines, "counters": {k: v for k, v in sorted(agg.items())}}
        json.dump(rec, open(args.out, "w"), indent=1)
        print("wrote", args.out, "bytes/launch %.4g" % rec["hbm_bytes_per_launch"])


if __name__ == "__main__":
    main()
