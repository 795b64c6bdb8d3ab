#!/usr/bin/env python3
"""Debug probe for the MSM window parts: n = 1 term, c = 4 (W = 65): reads the
top part's Horner accumulator from the workspace and compares it (and the
result) with the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import pairing_amd.device as pdev  # noqa: E402
from oracle import binding as o  # noqa: E402

R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
rng = np.random.default_rng(5)
a = int(rng.integers(1, 1 << 62))
s = int.from_bytes(rng.bytes(32), "little") % R


def sc(v):
    return np.array([[(v >> (64 * k)) & ((1 << 64) - 1) for k in range(4)]], dtype=np.uint64)


P = o.g1_mul_generator(sc(a))
c, W, B = 4, 65, 8
d, carry = [], 0
for w in range(W):
    raw = ((s >> (w * c)) & 15 if w * c < 256 else 0) + carry
    if raw > B:
        d.append(raw - 16); carry = 1
    else:
        d.append(raw); carry = 0
assert sum(x << (c * w) for w, x in enumerate(d)) == s
parts = int(os.environ.get("PA_MSM_PARTS", "2"))
wl = [W * (parts - 1 - q) // parts for q in range(parts)]
print("part lows", wl)
ws = pdev.multiexp_workspace(1, 1, "cuda")
out = torch.zeros((1, 18), dtype=torch.int64, device="cuda")
pdev.multiexp(1, torch.from_numpy(P.view(np.int64)).cuda(), torch.from_numpy(sc(s).view(np.int64)).cuda(), out, ws)
torch.cuda.synchronize()
got = out.cpu().numpy().view(np.uint64)
exp = o.g1_mul_generator(sc(a * s % R))
print("result ok:", bool((o.g1_into_affine(got) == exp).all()))
hb = ws.cpu().numpy()
off = hb.size - 1280
hacc = hb[off:off + 8 * 18 * 8].view(np.uint64).reshape(8, 18)
hi = W
for q in range(parts - 1):
    lo = wl[q]
    k = sum(d[w] << (c * (w - lo)) for w in range(lo, W)) % R
    e = o.g1_mul_generator(sc(a * k % R))
    g = o.g1_into_affine(hacc[q:q + 1].copy())
    print("leg", q, "windows [%d, %d)" % (lo, hi), "ok:", bool((g == e).all()), "z words", hacc[q, 12:14])
    hi = lo
