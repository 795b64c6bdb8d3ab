#!/usr/bin/env python3
"""Latency of small pairing batches (the verifier shape, mod.rs:49-95):
multi_pairing over n pairs and n independent pairings, through the
device-resident entry points (inputs in HBM; HIP events on the launch
stream), for the cooperative one-wave-per-pairing kernels and the one-lane
generated kernels.  DESIGN.md section 5."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
import pairing_amd  # noqa: E402
import pairing_amd.device as pdev  # noqa: E402


def timed(fn, reps=5):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


sizes = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 16, 64, 256, 1024, 2048, 4096]
VARIANTS = ((2, "coop4"), (4, "coop1"), (3, "one-lane"))
if os.environ.get("COOP_LAT_VARIANTS"):   # e.g. "1,3": lane pairs vs one lane for mid-size batches
    names = {0: "default", 1: "lane-pair", 2: "coop4", 3: "one-lane", 4: "coop1", 5: "lane-group"}
    VARIANTS = tuple((int(v), names[int(v)]) for v in os.environ["COOP_LAT_VARIANTS"].split(","))
for variant, name in VARIANTS:
    pairing_amd.set_pairing_kernel(variant)
    for n in sizes:
        p_np, q_np = bench.make_pairs(n, 0, seed=5)
        p = torch.from_numpy(p_np.view(np.int64)).cuda()
        q = torch.from_numpy(q_np.view(np.int64)).cuda()
        out = pdev.empty_records(n, 72, "cuda")
        scratch = pdev.empty_records(n, 72, "cuda")
        ms = timed(lambda: pdev.pairing(p, q, out, scratch))
        ml = timed(lambda: pdev.miller_loop(p, q, scratch))
        fe = timed(lambda: pdev.final_exponentiation(scratch, out))
        print("%-8s n=%5d  pairing batch %8.3f ms (ML %7.3f, FE %7.3f)  -> %9.0f pairings/s"
              % (name, n, ms, ml, fe, n / ms * 1e3), flush=True)
pairing_amd.set_pairing_kernel(0)
for n in (1, 2, 4, 16, 64, 256):
    p_np, q_np = bench.make_pairs(n, 0, seed=9)
    import time
    pairing_amd.multi_pairing(p_np, q_np)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        pairing_amd.multi_pairing(p_np, q_np)
        ts.append(time.perf_counter() - t0)
    print("default  multi_pairing n=%d (host buffers, includes copies): %.3f ms" % (n, sorted(ts)[2] * 1e3),
          flush=True)
