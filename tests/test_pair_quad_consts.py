"""Constants of the lane-group pairing kernels checked on the CPU (no GPU)."""
import os
import re

from helpers import Q

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_inversion_fix_constant_is_r_prime_cubed():
    """pair_quad.h kPqInvFix: the 28-bit limbs of R'^3 mod q (R' = 2^392), the
    factor that turns the binary GCD's plain inverse of x R' into x^-1 R'"""
    with open(os.path.join(ROOT, "pairing_amd", "csrc", "pair_quad.h")) as f:
        src = f.read()
    body = re.search(r"kPqInvFix\[14\] = \{(.*?)\};", src, re.S).group(1)
    limbs28 = [int(x.rstrip("u"), 16) for x in re.findall(r"0x[0-9a-fA-F]+u", body)]
    assert len(limbs28) == 14 and all(v < (1 << 28) for v in limbs28)
    assert sum(v << (28 * i) for i, v in enumerate(limbs28)) == pow(1 << 392, 3, Q)
