#!/usr/bin/env python3
"""Latency of compressed-point decoding (with subgroup checks) for small and
large batches through the host entry points (pairing_amd.g{1,2}_decode): the
verifier-shape cost of decoding a proof's points.  DESIGN.md section 9."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import pairing_amd  # noqa: E402

for n in (1, 2, 16, 1024, 65536):
    p_np, q_np = bench.make_pairs(n, 0, seed=13)
    e1, e2 = pairing_amd.g1_encode(p_np, True), pairing_amd.g2_encode(q_np, True)
    for name, fn, enc in (("g1", pairing_amd.g1_decode, e1), ("g2", pairing_amd.g2_decode, e2)):
        fn(enc, True)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            fn(enc, True)
            ts.append(time.perf_counter() - t0)
        print("%s decode n=%6d (host buffers, includes copies): %.3f ms" % (name, n, sorted(ts)[2] * 1e3),
              flush=True)
