#!/usr/bin/env python3
"""Summarise rocprofv3 output databases (kernel trace / PMC) into the small
text files committed under profiles/.

  tools/prof_summary.py kernels DB [DB...]        -> per-kernel stats table
  tools/prof_summary.py pmc DB COUNTER            -> per-kernel counter mean per dispatch
"""
import sqlite3
import sys


def kernels(paths):
    rows = {}
    meta = {}
    for p in paths:
        c = sqlite3.connect(p)
        for name, dur, vgpr, agpr, sgpr, scratch, gx, wx in c.execute(
                "select name, duration, vgpr_count, accum_vgpr_count, sgpr_count, scratch_size, grid_x, "
                "workgroup_x from kernels"):
            rows.setdefault(name, []).append(dur)
            meta[name] = (vgpr, agpr, sgpr, scratch, gx, wx)
    total = sum(sum(v) for v in rows.values())
    out = ["| kernel | calls | avg_us | min_us | max_us | share | vgpr | agpr | sgpr | scratch_B/lane | grid | wg |",
           "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for name, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        m = meta[name]
        out.append("| %s | %d | %.1f | %.1f | %.1f | %.1f%% | %s | %s | %s | %s | %s | %s |" % (
            name.replace("(anonymous namespace)::", "").split("(")[0], len(v), sum(v) / len(v) / 1e3, min(v) / 1e3, max(v) / 1e3,
            100.0 * sum(v) / total if total else 0, m[0], m[1], m[2], m[3], m[4], m[5]))
    return "\n".join(out)


def pmc(path, counter):
    c = sqlite3.connect(path)
    q = ("select k.name, e.value from pmc_events e join kernels k on e.kernel_id = k.kernel_id and "
         "e.dispatch_id = k.dispatch_id where e.counter_name = ?")
    try:
        rows = list(c.execute(q, (counter,)))
    except sqlite3.OperationalError:
        rows = []
    if not rows:  # schema fallback: the counters_collection view
        cur = c.execute("select * from counters_collection")
        cols = [d[0] for d in cur.description]
        rows = []
        for r in cur:
            d = dict(zip(cols, r))
            if d.get("counter_name") == counter:
                rows.append((d.get("kernel_name") or d.get("name"), d.get("value") or d.get("counter_value")))
    acc = {}
    for name, val in rows:
        acc.setdefault(name, []).append(float(val))
    out = ["| kernel | dispatches | %s mean/dispatch |" % counter, "|---|---|---|"]
    for name, v in sorted(acc.items()):
        out.append("| %s | %d | %.1f |" % (str(name).replace("(anonymous namespace)::", "").split("(")[0], len(v), sum(v) / len(v)))
    return "\n".join(out)


if __name__ == "__main__":
    if sys.argv[1] == "kernels":
        print(kernels(sys.argv[2:]))
    elif sys.argv[1] == "pmc":
        print(pmc(sys.argv[2], sys.argv[3]))
