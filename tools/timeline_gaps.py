#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel + memory-copy trace: every pairing kernel
and copy in start order with its queue, duration and the idle gap of the
compute pipe before it (host-boundary analysis).

  tools/timeline_gaps.py DB [--last N]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 40
    c = sqlite3.connect(db)
    ev = [("K", n, q, s, e) for n, q, s, e in c.execute("select name, queue_id, start, end from kernels")]
    try:
        ev += [("C", d, q, s, e) for d, q, s, e in c.execute("select direction, queue_id, start, end from memory_copies")]
    except sqlite3.Error:
        pass
    ev.sort(key=lambda x: x[3])
    ev = ev[-last:]
    t0 = ev[0][3]
    busy_end = None
    for kind, name, q, s, e in ev:
        gap = ""
        if kind == "K" and name.startswith("pa_gen"):
            if busy_end is not None:
                gap = "gap %.3f ms" % ((s - busy_end) / 1e6) if s > busy_end else "overlap"
            busy_end = e if busy_end is None else max(busy_end, e)
        print("%s %-28s q%-3s start %9.3f ms  dur %8.3f ms  %s" % (kind, str(name)[:28], q, (s - t0) / 1e6,
                                                                (e - s) / 1e6, gap))


if __name__ == "__main__":
    main()
