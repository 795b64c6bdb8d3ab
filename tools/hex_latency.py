#!/usr/bin/env python3
"""Latency of a dependent product chain in ONE wave: lane quads (coop_quad.h,
16 values per wave) vs 16-lane rows (coop_hex.h, 4 values per wave); the
test code object's coop_chain_probe kernel.  Prints ns per product level.

  python tools/hex_latency.py [iters]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import hipmod  # noqa: E402

CO = os.path.join(ROOT, "pairing_amd", "lib", "test", "coop_quad_unit.hsaco")
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
for mode, name in ((0, "quad (4 lanes / value)"), (1, "hex (16 lanes / value)")):
    best = None
    for rep in range(3):
        out = torch.zeros(80, dtype=torch.int32, device="cuda")
        hipmod.launch_kernel(CO, "coop_chain_probe", [(ctypes.c_uint64, out.data_ptr()), (ctypes.c_uint32, mode),
                                                       (ctypes.c_uint32, iters)], 1, 64)
        torch.cuda.synchronize()
        o = out.cpu().numpy().view(np.uint32)
        best = o[:2].copy() if best is None or o[0] < best[0] else best
    print("%-24s %8.1f ns per product level  (%6.0f shader clk)" % (name, best[0] * 10.0 / iters, best[1] / iters),
          flush=True)
