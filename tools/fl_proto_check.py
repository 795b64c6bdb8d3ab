#!/usr/bin/env python3
"""Check the Fl leaves (tools/gen_fl.py) on the GPU against Python integers,
including worst-case limb bounds, and time them against the 32-bit-word
multiply.  Usage: python tools/fl_proto_check.py path/to/fl_proto.so"""
import ctypes
import random
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from gen_consts import Q  # noqa: E402
from gen_fl import NL, LB, MASK, limbs, sub_constant  # noqa: E402

RL = 1 << (NL * LB)
RINV = pow(RL, -1, Q)
lib = ctypes.CDLL(sys.argv[1])
P = ctypes.c_void_p


def val(l):
    return sum(int(x) << (LB * i) for i, x in enumerate(l))


def lazy(u, rng):
    """limb-wise sum of u normalised values < 2q (bound u)"""
    acc = [0] * NL
    for _ in range(u):
        x = limbs(rng.randrange(2 * Q))
        acc = [a + b for a, b in zip(acc, x)]
    return acc


def maxed(u):
    return [u * MASK] * NL


def raw(op, rows):
    n = len(rows[0])
    arrs = [np.array(r, dtype=np.uint32).reshape(n, NL) for r in rows]
    while len(arrs) < 4:
        arrs.append(np.zeros((n, NL), np.uint32))
    out = np.zeros((n, NL), np.uint32)
    rc = lib.flp_raw(op, *[P(a.ctypes.data) for a in arrs], P(out.ctypes.data), n)
    assert rc == 0, rc
    return out


def check_products(name, op, cases, exact_bound=True):
    bad = 0
    for args, out in zip(zip(*cases), raw(op, cases)):
        vs = [val(a) for a in args]
        if op == 0:
            want = vs[0] * vs[1]
        elif op == 1:
            want = vs[0] * vs[1] + vs[2] * vs[3]
        else:
            want = vs[0] * vs[0]
        got = val(out)
        ok = (got - want * RINV) % Q == 0
        if exact_bound:
            ok = ok and got < 2 * Q and all(int(x) <= MASK for x in out)
        bad += not ok
    print("%-40s %d cases  %s" % (name, len(cases[0]), "OK" if bad == 0 else "FAIL %d" % bad))
    return bad


def main():
    rng = random.Random(7)
    bad = 0
    n = 512
    for ua, ub in [(1, 1), (1, 16), (16, 1), (4, 4), (3, 5), (2, 8)]:
        bad += check_products("mul u=(%d,%d) lazy" % (ua, ub), 0,
                              [[lazy(ua, rng) for _ in range(n)], [lazy(ub, rng) for _ in range(n)]])
        bad += check_products("mul u=(%d,%d) max limbs (congruence)" % (ua, ub), 0,
                              [[maxed(ua)] * 4, [maxed(ub)] * 4], exact_bound=False)
    for us in [(1, 1, 1, 1), (4, 2, 3, 3), (1, 8, 2, 4), (2, 2, 2, 2)]:
        bad += check_products("sop2 u=%s lazy" % (us,), 1, [[lazy(u, rng) for _ in range(n)] for u in us])
        bad += check_products("sop2 u=%s max limbs (congruence)" % (us,), 1, [[maxed(u)] * 4 for u in us],
                              exact_bound=False)
    for u in (1, 2, 3):
        bad += check_products("sqr u=%d lazy" % u, 2, [[lazy(u, rng) for _ in range(n)]])
        bad += check_products("sqr u=%d max limbs (congruence)" % u, 2, [[maxed(u)] * 4], exact_bound=False)
    # sub constants: a + C - b stays non-negative, value == a - b mod q
    for ub in range(1, 9):
        c, uc = sub_constant(ub)
        assert val(c) % Q == 0 and all(ci >= ub * MASK for ci in c[:-1])
    # ABI conversion round trip: canonical R=2^384 in, canonical out
    m = 4096
    a = [rng.randrange(Q) for _ in range(m)]
    b = [rng.randrange(Q) for _ in range(m)]
    a[0], b[0] = Q - 1, Q - 1
    a[1], b[1] = 0, 5
    enc = lambda xs: np.array([[(x >> (64 * i)) & (2**64 - 1) for i in range(6)] for x in xs], dtype=np.uint64)
    A, B = enc(a), enc(b)
    O = np.zeros_like(A)
    assert lib.flp_abi(P(A.ctypes.data), P(B.ctypes.data), P(O.ctypes.data), m) == 0
    ri = pow(2, -384, Q)
    got = [sum(int(O[j, i]) << (64 * i) for i in range(6)) for j in range(m)]
    badabi = sum(g != (x * y * ri) % Q for g, x, y in zip(got, a, b))
    print("%-40s %d cases  %s" % ("ABI mont mul (R=2^384) via Fl", m, "OK" if badabi == 0 else "FAIL %d" % badabi))
    bad += badabi
    # throughput
    lib.flp_time.restype = ctypes.c_float
    nn = 65536
    X = enc([rng.randrange(Q) for _ in range(nn)])
    iters = 2000
    for op, nm in [(0, "fq_mul 12x32 FIPS (current)"), (1, "fl_mul_leaf 14x28"), (2, "fl_sqr_leaf 14x28")]:
        ms = lib.flp_time(op, P(X.ctypes.data), nn, iters)
        print("%-32s %8.3f ms  %.3f ns/product/lane-batch  %.2f G products/s" % (
            nm, ms, ms * 1e6 / iters, nn * iters / (ms * 1e-3) / 1e9))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
