"""Print the kernel timeline (start/end relative to a marker kernel, per
stream) around an occurrence of the marker (default the last) from a
rocprofv3 --kernel-trace rocpd database:
python tools/kernel_timeline.py DB MARKER [N [OCCURRENCE]]"""
import sqlite3
import sys

db, marker = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
occ = int(sys.argv[4]) if len(sys.argv) > 4 else -1
c = sqlite3.connect(db)
rows = list(c.execute("select name, start, end, stream_id from kernels order by start"))
idx = [i for i, r in enumerate(rows) if marker in r[0]][occ]
base = rows[idx][1]
for r in rows[max(idx - 2, 0):idx + n]:
    print(f"{r[0][:44]:44s} {(r[1] - base) / 1e3:9.1f} {(r[2] - base) / 1e3:9.1f} dur {(r[2] - r[1]) / 1e3:8.1f} s{r[3]}")
