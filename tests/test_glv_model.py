"""CPU model of config 3's GLV form (kernels_curve.hip), with the constants
read from the kernel source so the ones tested are the ones shipped:

* phi(x, y) = (beta x, y) acts on G1 as -x^2 (the identity k_g1_glv_check
  tests per base), for the BLS12-381 generator and a random multiple of it,
  and not on a point outside G1 (so such a base takes the fallback);
* glv_split's Barrett step: for every 256-bit s, q = floor(floor(s / 2^127) m
  / 2^129) and rem = s - q x^2 satisfy 0 <= rem < 2^129, q < 2^129, and both
  recode into 17 signed base-256 digits with no carry out (the 17 windows
  k_g1_glv_mul walks), at the edges and on random values;
* the average number of nonzero digits bench.py prices the roofline with."""
import os
import re

import numpy as np

import decode_cases as D
from helpers import Q, R_ORDER

SRC = os.path.join(os.path.dirname(__file__), "..", "pairing_amd", "csrc", "kernels_curve.hip")
X_ABS = 0xd201000000010000
X2 = X_ABS * X_ABS
G1X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1


def _src():
    with open(SRC) as f:
        return f.read()


def _words(body):
    return [int(w, 16) for w in re.findall(r"0x([0-9a-fA-F]+)", body)]


def _beta():
    m = re.search(r"kGlvBeta\[6\]\s*=\s*\{([^}]*)\}", _src())
    ws = _words(m.group(1))
    mont = sum(w << (64 * i) for i, w in enumerate(ws))
    return mont * pow(2, -384, Q) % Q   # Montgomery R = 2^384 -> integer


def _barrett_m():
    m = re.search(r"constexpr uint64_t m\[3\]\s*=\s*\{([^}]*)\}", _src())
    ws = [int(t.strip().rstrip("ull").rstrip("u"), 0) for t in m.group(1).split(",")]
    return sum(w << (64 * i) for i, w in enumerate(ws))


def _x2_words():
    m = re.search(r"kX2Lo\s*=\s*0x([0-9a-fA-F]+)ull,\s*kX2Hi\s*=\s*0x([0-9a-fA-F]+)ull", _src())
    return int(m.group(1), 16) | int(m.group(2), 16) << 64


def _split(s, m):
    q = ((s >> 127) * m) >> 129
    return q, s - q * X2


def _digits(v, windows=17):
    out, carry = [], 0
    for w in range(windows):
        d = carry + ((v >> (8 * w)) & 0xff)
        carry = 1 if d > 128 else 0
        out.append(d - 256 if d > 128 else d)
    return out, carry


def test_constants_match_the_parameter():
    assert _x2_words() == X2
    assert _barrett_m() == (1 << 256) // X2
    beta = _beta()
    assert beta != 1 and pow(beta, 3, Q) == 1


def test_phi_is_minus_x_squared_on_g1_only():
    F = D._f1()
    beta = _beta()
    g = (G1X, G1Y)
    rng = np.random.default_rng(80)
    p = D._ec_mul(F, g, int(rng.integers(1, 1 << 62)) << 64 | int(rng.integers(1, 1 << 62)))
    for P in (g, p):
        lhs = (beta * P[0] % Q, P[1])
        mx = D._ec_mul(F, P, X2)
        assert lhs == (mx[0], (-mx[1]) % Q)
    pts, truth = D.subgroup_points(1, seed=81, n=2)
    for P, t in zip(pts, truth):
        mx = D._ec_mul(F, P, X2)
        ok = mx is not None and (beta * P[0] % Q, P[1]) == (mx[0], (-mx[1]) % Q)
        assert ok == t


def test_barrett_split_bounds_and_digits():
    m = _barrett_m()
    edges = [0, 1, X2 - 1, X2, X2 + 1, 2 * X2 - 1, (1 << 128) - 1, 1 << 128, (1 << 129) * X2 // 2,
             R_ORDER - 1, R_ORDER, (1 << 255) - 1, (1 << 256) - 1, ((1 << 256) - 1) // X2 * X2,
             ((1 << 256) - 1) // X2 * X2 - 1]
    rng = np.random.default_rng(82)
    rand = [int.from_bytes(rng.bytes(32), "little") for _ in range(3000)]
    for s in edges + rand:
        q, rem = _split(s, m)
        assert q * X2 + rem == s
        assert 0 <= rem < (1 << 129) and 0 <= q < (1 << 129)
        for v in (q, rem):
            ds, carry = _digits(v)
            assert carry == 0 and sum(d << (8 * w) for w, d in enumerate(ds)) == v


def test_nonzero_digit_average_priced_by_bench():
    m = _barrett_m()
    rng = np.random.default_rng(83)
    tot = 0
    n = 4000
    for _ in range(n):
        s = int.from_bytes(rng.bytes(32), "little") % R_ORDER
        q, rem = _split(s, m)
        tot += sum(d != 0 for d in _digits(rem)[0]) + sum(d != 0 for d in _digits(q)[0])
    assert abs(tot / n - 32.77) < 0.1
