#!/usr/bin/env python3
"""G2 fixed-base (Wnaf::base(g, n).scalar(s_i)) timing probe: device-resident
pa_g2_wnaf_fixed_base_device (table build + multiply), HIP events, median of 5;
a sample checked against the oracle's G2 wNAF.  PA_LIB_PATH selects another
build for A/B runs.

  python tools/g2_comb_probe.py [n ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import pairing_amd.device as pdev  # noqa: E402
from oracle import binding as o  # noqa: E402

for n in [int(x) for x in sys.argv[1:]] or [1 << 16]:
    rng = np.random.default_rng(n)
    s = rng.integers(0, 1 << 63, size=(n, 4), dtype=np.uint64)
    base = o.g2_from_affine(o.g2_mul_generator(np.array([[12345, 0, 0, 0]], dtype=np.uint64)))
    db = torch.from_numpy(base.view(np.int64)).cuda()
    ds = torch.from_numpy(s.view(np.int64)).cuda()
    out = pdev.empty_records(n, 36, "cuda")
    table, ws = pdev.g2_fixed_base_buffers("cuda")
    st = torch.cuda.current_stream()
    ts = []
    for r in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        pdev.g2_wnaf_fixed_base(db, ds, out, table, ws)
        e1.record(st)
        torch.cuda.synchronize()
        if r >= 2:
            ts.append(e0.elapsed_time(e1))
    k = 64
    got = out[:k].cpu().numpy().view(np.uint64)
    exp = o.g2_wnaf_fixed_base(base, s[:k])
    ok = bool(o.g2_eq(got, exp).all())
    ms = sorted(ts)[len(ts) // 2]
    print("G2 fixed base n=%d  %.3f ms  %.2f M points/s  sample ok=%s  lib=%s" % (
        n, ms, n / ms / 1e3, ok, os.path.basename(os.path.dirname(os.environ.get("PA_LIB_PATH", "default")))),
        flush=True)
