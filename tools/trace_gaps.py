"""Per-kernel totals and GPU idle time over the last timed step(s) of a rocprofv3 kernel-trace CSV:
the busy union of all dispatches between the first and the last dispatch of the window, the idle
gaps longer than a threshold, and the kernels' summed durations.

    python tools/trace_gaps.py run_kernel_trace.csv [window_start_kernel] [n_last]
"""
import csv
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "lr_screen_kernel"
nlast = int(sys.argv[3]) if len(sys.argv) > 3 else 98
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
idx = [k for k, r in enumerate(rows) if pat in r[2]]
sel = idx[-nlast:]
lo, hi = rows[sel[0]][0], rows[sel[-1]][1]
win = [r for r in rows if r[1] > lo and r[0] < hi]
busy, gaps = 0, []
cs, ce = win[0][0], win[0][1]
for s, e, _ in win[1:]:
    if s > ce:
        busy += ce - cs
        gaps.append(s - ce)
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print("window %.2f ms  busy %.2f ms  idle %.2f ms  (%d gaps > 20 us: %.2f ms)" % (
    (hi - lo) / 1e6, busy / 1e6, (hi - lo - busy) / 1e6, sum(g > 20000 for g in gaps),
    sum(g for g in gaps if g > 20000) / 1e6))
tot = {}
for s, e, n in win:
    k = n.split("(")[0][-60:]
    tot.setdefault(k, [0, 0.0])
    tot[k][0] += 1
    tot[k][1] += (min(e, hi) - max(s, lo)) / 1e6
for k, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1])[:14]:
    print("%-62s %5d %9.2f ms" % (k, c, t))
