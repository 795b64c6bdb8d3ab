#!/usr/bin/env python3
"""Write tests/golden/bench_points.npz: 256 random G1 and 256 random G2 affine
points (k*G for seeded random k < r) in the ABI layout, the synthetic input
pool bench.py draws its batches from.  Generated once here with the oracle
so that bench.py itself never runs oracle code outside its cpu_baseline leg.

The pairing kernels' control flow does not depend on the point values (only
on the infinity flags), so a batch tiled from 256 x 256 distinct combinations
costs the same as 2^16 fresh points."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import random_scalars, rng  # noqa: E402
from oracle import binding as oracle  # noqa: E402


def main():
    g = rng(20261015)
    s1 = random_scalars(g, 256)
    s2 = random_scalars(g, 256)
    g1 = oracle.g1_mul_generator(s1, 8)
    g2 = oracle.g2_mul_generator(s2, 8)
    out = os.path.join(ROOT, "tests", "golden", "bench_points.npz")
    np.savez_compressed(out, g1=g1, g2=g2, s1=s1, s2=s2)
    print("wrote", out)


if __name__ == "__main__":
    main()
