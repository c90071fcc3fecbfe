"""Kernel time of the last timed scan step from a rocprofv3 --kernel-trace CSV: the window from the
first prefilter pass after the previous step's refine (or the first of the last `launches` passes,
when given) to the last refine, its busy union and per-kernel totals, and the time in which each
kernel ran alone.   python tools/step_timeline.py run_kernel_trace.csv [launches]"""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return re.sub(r"^(void )?(gmat::)?(epi::)?", "", name).split("(")[0][:48]


def main():
    path = sys.argv[1]
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in csv.DictReader(open(path)))
    rf = [k for k, e in enumerate(ev) if e[2].startswith(("refine_kernel", "refine8_side_kernel", "refine8_fin_kernel"))]
    if any(ev[k][2].startswith("refine8_fin_kernel") for k in rf):  # round 5: the finish kernel ends a scan
        rf = [k for k in rf if ev[k][2].startswith("refine8_fin_kernel")]
    pf = [k for k, e in enumerate(ev) if e[2].startswith(("prefilter_pass", "prefilter_cov"))]
    if len(sys.argv) > 2:
        pf = pf[-int(sys.argv[2]):]
    elif len(rf) >= 2:  # the last step: the passes after the previous step's refine
        pf = [k for k in pf if ev[k][0] >= ev[rf[-2]][1]]
    lo, hi = ev[pf[0]][0], max(ev[rf[-1]][1], ev[pf[-1]][1])
    win = [(max(s, lo), min(e, hi), n) for s, e, n in ev if e > lo and s < hi]
    pts = sorted({t for s, e, _ in win for t in (s, e)})
    busy = 0
    alone = {}
    for a, b in zip(pts, pts[1:]):
        run = [n for s, e, n in win if s <= a and e >= b]
        if run:
            busy += b - a
        if len(set(run)) == 1:
            alone[run[0]] = alone.get(run[0], 0) + b - a
    print("window %.2f ms, busy %.2f ms, idle %.2f ms" % ((hi - lo) / 1e6, busy / 1e6, (hi - lo - busy) / 1e6))
    tot = {}
    for s, e, n in win:
        c, t = tot.get(n, (0, 0))
        tot[n] = (c + 1, t + e - s)
    print("%-48s %6s %10s %10s" % ("kernel", "calls", "sum ms", "alone ms"))
    for n, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1]):
        print("%-48s %6d %10.2f %10.2f" % (n, c, t / 1e6, alone.get(n, 0) / 1e6))


if __name__ == "__main__":
    main()
