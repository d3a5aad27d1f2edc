"""Per-kernel summary of a rocprofv3 results database (rocpd sqlite)."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
q = ("select name, count(*), avg(end-start), min(end-start), sum(end-start) from kernels "
     "group by name order by sum(end-start) desc limit 12")
print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>8s} {'min_us':>8s} {'total_ms':>9s}")
for name, n, avg, mn, tot in c.execute(q):
    print(f"{name[:70]:70s} {n:6d} {avg / 1e3:8.2f} {mn / 1e3:8.2f} {tot / 1e6:9.3f}")
