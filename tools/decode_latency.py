#!/usr/bin/env python3
"""Latency of compressed-point decoding (with subgroup checks) by batch size,
for both decode kernels (pa_set_decode_kernel: 1 = one lane per record, 2 =
one record per group of lane quads): device-resident (HIP events on the
launch stream) and through the host entry points (pairing_amd.g{1,2}_decode,
copies included).  The verifier-shape cost of decoding a proof's points;
DESIGN.md section 4.

  python tools/decode_latency.py [n ...]     (DECODE_VARIANTS=1,2 by default)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
import pairing_amd  # noqa: E402
import pairing_amd.device as pdev  # noqa: E402


def dev_ms(group, enc_t, n, reps=7):
    w = 13 if group == 1 else 25
    out = torch.empty((n, w), dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(2):
        pdev.decode(group, enc_t, True, True, out, st)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        pdev.decode(group, enc_t, True, True, out, st)
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


sizes = [int(x) for x in sys.argv[1:]] or [1, 2, 16, 256, 1024, 4096, 16384, 65536]
variants = [int(v) for v in os.environ.get("DECODE_VARIANTS", "1,2").split(",")]
for v in variants:
    pairing_amd.set_decode_kernel(v)
    name = {0: "default", 1: "one-lane", 2: "quad"}[v]
    for n in sizes:
        p_np, q_np = bench.make_pairs(n, 0, seed=13)
        e1, e2 = pairing_amd.g1_encode(p_np, True), pairing_amd.g2_encode(q_np, True)
        for g, fn, enc in ((1, pairing_amd.g1_decode, e1), (2, pairing_amd.g2_decode, e2)):
            d = dev_ms(g, torch.from_numpy(np.ascontiguousarray(enc)).cuda(), n)
            fn(enc, True)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                fn(enc, True)
                ts.append(time.perf_counter() - t0)
            print("%-8s g%d decode n=%6d  device %8.3f ms  host buffers %8.3f ms" % (name, g, n, d, sorted(ts)[2] * 1e3),
                  flush=True)
pairing_amd.set_decode_kernel(0)
