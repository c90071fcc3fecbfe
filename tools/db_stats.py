"""Per-kernel stats (calls, total/avg µs) from a rocprofv3 rocpd SQLite database."""
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
q = """select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start)
       from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
       group by s.kernel_name order by sum(d.end - d.start) desc"""
print("%-70s %6s %12s %10s" % ("kernel", "calls", "total_ms", "avg_us"))
for name, n, tot, avg in con.execute(q).fetchall()[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print("%-70s %6d %12.3f %10.1f" % (name[:70], n, tot / 1e6, avg / 1e3))
