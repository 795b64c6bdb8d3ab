#!/usr/bin/env python3
"""One pairing batch per kernel variant, for rocprofv3 --pmc passes
(why two co-resident lane-pair waves per SIMD add no
throughput).  Usage: tools/pair_pmc.py N VARIANT [REPS]

Runs the Miller loop and the final exponentiation of N pairings (inputs
resident in HBM, the bench's points) once as warm-up and REPS times more, on
the device entry points, with pa_set_pairing_kernel(VARIANT): 1 = lane pairs,
3 = one lane per pairing.  Prints the HIP-event time of each launch."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
import pairing_amd  # noqa: E402
import pairing_amd.device as pdev  # noqa: E402

n = int(sys.argv[1])
variant = int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
pairing_amd.set_pairing_kernel(variant)
p_np, q_np = bench.make_pairs(n, 0, seed=5)
p = torch.from_numpy(p_np.view(np.int64)).cuda()
q = torch.from_numpy(q_np.view(np.int64)).cuda()
f = pdev.empty_records(n, 72, "cuda")
out = pdev.empty_records(n, 72, "cuda")
s = torch.cuda.current_stream()
for r in range(reps + 1):
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record(s)
    pdev.miller_loop(p, q, f)
    e[1].record(s)
    pdev.final_exponentiation(f, out)
    e[2].record(s)
    torch.cuda.synchronize()
    print("variant %d n=%d %s ML %.3f ms FE %.3f ms" % (variant, n, "warm-up" if r == 0 else "run",
                                                        e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2])),
          flush=True)
