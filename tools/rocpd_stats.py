"""Per-kernel summary from a rocprofv3 rocpd database (run_results.db):
usage rocpd_stats.py DB [divisor] [top]; divisor = frames/iterations."""
import sqlite3
import sys

db = sys.argv[1]
div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), sum(duration), avg(duration) from kernels group by name "
                 "order by sum(duration) desc").fetchall()
tot = sum(r[2] for r in rows)
n = sum(r[1] for r in rows)
span = c.execute("select max(end) - min(start) from kernels").fetchone()[0]
print(f"kernel time {tot / 1e3 / div:.1f} us/iter, launches {n / div:.1f}/iter, span {span / 1e3 / div:.1f} us/iter")
for r in rows[:top]:
    print(f"{r[2] / 1e3 / div:9.1f} us/iter {r[1] / div:7.1f}x {r[3] / 1e3:8.2f} us  {r[0][:100]}")
