"""Per-kernel summary of a rocprofv3 results database (rocpd sqlite).

usage: python tools/kstats.py RESULTS.db [--top N] [--steps S]
  --steps S also prints the per-step GPU busy time (sum of kernel time / S)."""
import argparse
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--top", type=int, default=12)
ap.add_argument("--steps", type=int, default=0)
a = ap.parse_args()
c = sqlite3.connect(a.db)
q = ("select name, count(*), avg(end-start), min(end-start), sum(end-start) from kernels "
     "group by name order by sum(end-start) desc limit ?")
print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>8s} {'min_us':>8s} {'total_ms':>9s}")
for name, n, avg, mn, tot in c.execute(q, (a.top,)):
    print(f"{name[:70]:70s} {n:6d} {avg / 1e3:8.2f} {mn / 1e3:8.2f} {tot / 1e6:9.3f}")
(total, n) = c.execute("select sum(end-start), count(*) from kernels").fetchone()
print(f"all kernels: {n} launches, {total / 1e6:.3f} ms")
if a.steps:
    print(f"per step: {n / a.steps:.1f} launches, {total / 1e3 / a.steps:.1f} us GPU busy")
