#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer boundary: pa_pairing_batch on host
arrays (pinned staging, H2D, fused Miller loop + final exponentiation, D2H,
copy-out), the bench's synthetic inputs.  Reports one caller at 2^16 and
2^17 pairings (the latter pipelines two device-filling chunks) and two host
threads calling at once (each its own stream: one thread's transfers overlap
the other's kernels).  DESIGN.md section 7."""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (make_pairs)
import pairing_amd  # noqa: E402


def median_time(fn, reps=5):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


pairing_amd.set_device(0)
n = 1 << 16
p, q = bench.make_pairs(2 * n, 0)
out = np.empty((2 * n, 72), np.uint64)
pairing_amd.pairing(p[:1024], q[:1024])  # warm-up (code objects, contexts)
pieces = os.environ.get("PA_PIPELINE_PIECES", "1")
for m in (n, 2 * n):
    pairing_amd.pairing(p[:m], q[:m])
    t = median_time(lambda: pairing_amd.pairing(p[:m], q[:m]))
    print("one caller, n=%d, fresh result array: median %.2f ms -> %.0f pairings/s (bytes in %d, out %d; pieces %s)"
          % (m, t * 1e3, m / t, p[:m].nbytes + q[:m].nbytes, m * 576, pieces), flush=True)
    o = out[:m]
    pairing_amd.pairing(p[:m], q[:m], out=o)
    t = median_time(lambda: pairing_amd.pairing(p[:m], q[:m], out=o))
    print("one caller, n=%d, reused result array: median %.2f ms -> %.0f pairings/s (pieces %s)"
          % (m, t * 1e3, m / t, pieces), flush=True)
    if os.environ.get("PA_PIPELINE_TRACE") == "1":
        break


def worker(k, reps):
    for _ in range(reps):
        pairing_amd.pairing(p[k * n:(k + 1) * n], q[k * n:(k + 1) * n])


reps = 6
worker(0, 1)
th = [threading.Thread(target=worker, args=(k, reps)) for k in range(2)]
t0 = time.perf_counter()
for t in th:
    t.start()
for t in th:
    t.join()
t = time.perf_counter() - t0
print("two host threads, n=%d each, %d calls each: %.2f ms -> %.0f pairings/s aggregate"
      % (n, reps, t * 1e3, 2 * reps * n / t), flush=True)
