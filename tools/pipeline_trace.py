#!/usr/bin/env python3
"""One traced host-buffer pa_pairing_batch call (PA_PIPELINE_TRACE=1):
per-phase timestamps of the pinned-staging pipeline, for DESIGN.md's
boundary numbers."""
import os
import sys
import time

os.environ["PA_PIPELINE_TRACE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import pairing_amd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
p, q = bench.make_pairs(n, 0)
pairing_amd.pairing(p[:1024], q[:1024])
pairing_amd.pairing(p, q)
for _ in range(2):
    t0 = time.perf_counter()
    pairing_amd.pairing(p, q)
    print("call %.2f ms" % ((time.perf_counter() - t0) * 1e3), file=sys.stderr, flush=True)
