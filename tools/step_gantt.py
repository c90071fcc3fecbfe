"""The last timed scan step of a rocprofv3 --kernel-trace CSV as a list of kernel launches in start
order (queue, start / end in us from the step's first prefilter pass, duration), then the step's time
split by what ran: with a prefilter pass, with candidate kernels only, idle.
   python tools/step_gantt.py run_kernel_trace.csv"""
import csv
import sys

from step_timeline import short


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                 r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows)
    fin = [k for k, e in enumerate(ev) if e[2].startswith("refine8_fin_kernel")]
    pf = [k for k, e in enumerate(ev) if e[2].startswith(("prefilter_pass", "prefilter_cov"))]
    if len(fin) >= 2:
        pf = [k for k in pf if ev[k][0] >= ev[fin[-2]][1]]
    lo = ev[pf[0]][0]
    hi = max(ev[fin[-1]][1], ev[pf[-1]][1])
    win = [e for e in ev if e[1] > lo and e[0] < hi]
    for s, e, n, q in win:
        print("%-40s q%-4s %9.1f %9.1f %8.1f" % (n[:40], q, (s - lo) / 1e3, (e - lo) / 1e3, (e - s) / 1e3))
    pts = sorted({t for s, e, _, _ in win for t in (max(s, lo), min(e, hi))})
    with_pf = cand_only = idle = 0
    for a, b in zip(pts, pts[1:]):
        run = [n for s, e, n, _ in win if s <= a and e >= b]
        if any(n.startswith("prefilter") for n in run):
            with_pf += b - a
        elif run:
            cand_only += b - a
        else:
            idle += b - a
    print("window %.2f ms: a prefilter pass running %.2f ms, candidate kernels only %.2f ms, idle %.2f ms"
          % ((hi - lo) / 1e6, with_pf / 1e6, cand_only / 1e6, idle / 1e6))


if __name__ == "__main__":
    main()
