#!/usr/bin/env python3
"""G2 MSM timing probe (bench.py's msm line is G1): device-resident
pa_g2_multiexp_device over n random terms, HIP events on the launch stream,
median of 5; the result checked against the G1-free identity
sum s_i (a_i G2) = (sum s_i a_i) G2 through the oracle.

  python tools/msm_g2_probe.py [n ...]      (PA_MSM_G2_LAZY=0: the 12-word kernels)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import pairing_amd.device as pdev  # noqa: E402
from oracle import binding as o  # noqa: E402

R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


def scal(vals):
    return np.array([[(v >> (64 * k)) & ((1 << 64) - 1) for k in range(4)] for v in vals], dtype=np.uint64)


for n in [int(x) for x in sys.argv[1:]] or [1 << 16]:
    rng = np.random.default_rng(n)
    a = [int(x) for x in rng.integers(1, 1 << 62, n)]
    s = [int.from_bytes(rng.bytes(32), "little") % R for _ in range(n)]
    p = o.g2_mul_generator(scal(a), 16)
    dp = torch.from_numpy(p.view(np.int64)).cuda()
    ds = torch.from_numpy(scal(s).view(np.int64)).cuda()
    out = pdev.empty_records(1, 36, "cuda")
    ws = pdev.multiexp_workspace(2, n, "cuda")
    st = torch.cuda.current_stream()
    ts = []
    for r in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        pdev.multiexp(2, dp, ds, out, ws)
        e1.record(st)
        torch.cuda.synchronize()
        if r >= 2:
            ts.append(e0.elapsed_time(e1))
    tot = sum(x * y for x, y in zip(a, s)) % R
    ok = bool((o.g2_into_affine(out.cpu().numpy().view(np.uint64)) == o.g2_mul_generator(scal([tot]))).all())
    ms = sorted(ts)[len(ts) // 2]
    print("G2 MSM n=%d  lazy=%s  %.3f ms  %.2f M terms/s  ok=%s" % (n, os.environ.get("PA_MSM_G2_LAZY", "1"), ms,
                                                                   n / ms / 1e3, ok), flush=True)
