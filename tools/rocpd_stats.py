"""Per-kernel stats (calls, average / min / max us, share) from a rocprofv3
rocpd database, as a markdown table: python tools/rocpd_stats.py DB [TOP]"""
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
c = sqlite3.connect(db)
rows = list(c.execute("select name, count(*), avg(end - start), min(end - start), max(end - start), "
                      "sum(end - start) from kernels group by name order by sum(end - start) desc"))
total = sum(r[5] for r in rows)
print("| kernel | calls | avg_us | min_us | max_us | share |")
print("|---|---|---|---|---|---|")
for name, n, avg, mn, mx, tot in rows[:top]:
    print(f"| {name.split('(')[0][:70]} | {n} | {avg / 1e3:.1f} | {mn / 1e3:.1f} | {mx / 1e3:.1f} | {100 * tot / total:.1f}% |")
