"""Timeline summary of the last timed step from a rocprofv3 rocpd database: busy union, gaps,
per-kernel totals inside the window of the last `nscreen` screen launches."""
import sqlite3
import sys

db, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "screen_kernel")
nlast = int(sys.argv[3]) if len(sys.argv) > 3 else 98
con = sqlite3.connect(db)
rows = con.execute("""select d.start, d.end, s.kernel_name from rocpd_kernel_dispatch d
                      join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start""").fetchall()
idx = [k for k, r in enumerate(rows) if pat in r[2]]
sel = idx[-nlast:]
lo, hi = rows[sel[0]][0], rows[sel[-1]][1]
win = [r for r in rows if r[1] > lo and r[0] < hi]
iv = sorted((max(s, lo), min(e, hi)) for s, e, _ in win)
busy, (cs, ce) = 0, iv[0]
for s, e in iv[1:]:
    if s > ce:
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print("window %.2f ms  busy %.2f ms  idle %.2f ms" % ((hi - lo) / 1e6, busy / 1e6, (hi - lo - busy) / 1e6))
tot = {}
for s, e, n in win:
    k = n.split("(")[0][:60]
    tot.setdefault(k, [0, 0.0])
    tot[k][0] += 1
    tot[k][1] += (min(e, hi) - max(s, lo)) / 1e6
for k, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1])[:12]:
    print("%-62s %5d %9.2f ms" % (k, c, t))
