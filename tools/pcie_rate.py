#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer boundary: pa_pairing_batch on host
arrays (upload G1/G2 records, fused Miller loop + final exponentiation,
download Fq12), batch 2^16, the bench's synthetic inputs.  DESIGN.md §7."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (make_pairs)
import pairing_amd  # noqa: E402

n = 1 << 16
p, q = bench.make_pairs(n, 0)
pairing_amd.set_device(0)
pairing_amd.pairing(p[:1024], q[:1024])  # warm-up (code objects, allocations)
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    pairing_amd.pairing(p, q)
    ts.append(time.perf_counter() - t0)
t = sorted(ts)[len(ts) // 2]
print("host-buffer pa_pairing_batch, n=%d: median %.2f ms -> %.0f pairings/s (bytes in %d, out %d)"
      % (n, t * 1e3, n / t, p.nbytes + q.nbytes, n * 576))
