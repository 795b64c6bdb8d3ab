#!/usr/bin/env python3
"""Software-pipelined pairing batches (experiment): the Miller loop of batch
k + 1 on one stream while the final exponentiation of batch k runs on another,
so that with code objects built for two waves per SIMD (PGEN_TWO_WAVES=1,
256 registers per wave; PA_GEN_DIR=gpuvar/w2) an ML wave and an FE wave can
share each SIMD.  Prints ms per 2^16-pairing step, sequential vs pipelined.

  PA_GEN_DIR=$PWD/gpuvar/w2 PA_GEN_WS_SLOTS=160 python tools/pipe_probe.py"""
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

n = int(os.environ.get("PIPE_N", 1 << 16))
steps = 10
pairing_amd.set_pairing_kernel(3)   # one lane per pairing at every size
p_np, q_np = bench.make_pairs(n, 0, seed=1)
p = torch.from_numpy(p_np.view(np.int64)).cuda()
q = torch.from_numpy(q_np.view(np.int64)).cuda()
f = [pdev.empty_records(n, 72, "cuda") for _ in range(2)]
out = pdev.empty_records(n, 72, "cuda")
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()


def seq():
    for _ in range(steps):
        pdev.miller_loop(p, q, f[0], sa)
        pdev.final_exponentiation(f[0], out, None, sa)


def pipe():
    fe_done = [None, None]
    pdev.miller_loop(p, q, f[0], sa)
    for s in range(steps):
        ml_done = torch.cuda.Event()
        ml_done.record(sa)
        sb.wait_event(ml_done)
        pdev.final_exponentiation(f[s % 2], out, None, sb)
        e = torch.cuda.Event()
        e.record(sb)
        fe_done[s % 2] = e
        if s + 1 < steps:
            if fe_done[(s + 1) % 2] is not None:
                sa.wait_event(fe_done[(s + 1) % 2])
            pdev.miller_loop(p, q, f[(s + 1) % 2], sa)


for name, fn in (("sequential", seq), ("pipelined", pipe), ("sequential", seq), ("pipelined", pipe)):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    print("%-10s n=%d  %.3f ms per step  %.0f pairings/s" % (name, n, ms, n / ms * 1e3), flush=True)
# parity of the pipelined outputs on a sample
exp = pairing_amd.pairing(p_np[:64], q_np[:64])
got = out[:64].cpu().numpy().view(np.uint64)
print("sample parity:", bool(np.array_equal(got, exp)))
