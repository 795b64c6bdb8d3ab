#!/usr/bin/env python3
"""Fixture for the rare branch of Karabina decompression (tools/pgen/tower.py
kdec_numden): a cyclotomic-subgroup element f of Fq12 whose coordinate b0
(f = (a0 + a1 v + a2 v^2) + (b0 + b1 v + b2 v^2) w) is ZERO, so that
b1 = 2 a1 b2 / a2 instead of (3 a1^2 - 2 a2 + xi b2^2) / (4 b0).  Random
elements hit b0 = 0 with probability ~q^-2, so one is constructed:

  * every element of the cyclotomic subgroup G_{Phi_6}(q^2) is h^(q^2 + 1) for
    a unitary h (h conj(h) = 1), and the unitary h are (alpha + w) / (alpha - w)
    with alpha in Fq6;
  * along the line alpha(t) = alpha0 + t delta (t in Fq2, which the q^2-power
    Frobenius F fixes), f(t) = N(t) / D(t) with N = (alpha + w) F(alpha + w),
    D = (alpha - w) F(alpha - w) quadratic in t, so b0(f(t)) Norm(D(t)) =
    b0(N(t) adj(D(t))) =: P(t) is a polynomial of degree <= 12 over Fq2
    (adj(D) = F(D) F^2(D) ... F^5(D), Norm(D) = D adj(D) in Fq2);
  * P is interpolated from 13 evaluations and its roots in Fq2 are the factors
    of gcd(P, t^(q^2) - t) (Cantor-Zassenhaus for gcds of degree > 1).

The written element is checked to be unitary and in G_{Phi_6} by the Python
model (tests/pymodel.py: f^(q^4 - q^2 + 1) == 1).  Run from the repo root:
  python tests/golden/make_karabina_fixture.py  -> tests/golden/karabina_b0zero.json
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from pymodel import (F12ONE, f12conj, f12inv, f12mul, f12pow, f2add, f2inv, f2mul, f2sub)  # noqa: E402
from helpers import Q  # noqa: E402

Z2 = (0, 0)
O2 = (1, 0)


# ---- polynomials over Fq2 (lists of coefficients, low degree first) ----
def ptrim(a):
    a = list(a)
    while a and a[-1] == Z2:
        a.pop()
    return a


def pmul(a, b):
    if not a or not b:
        return []
    c = [Z2] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        for j, y in enumerate(b):
            c[i + j] = f2add(c[i + j], f2mul(x, y))
    return ptrim(c)


def pdivmod(a, b):
    a, b = ptrim(a), ptrim(b)
    inv = f2inv(b[-1])
    q = [Z2] * max(0, len(a) - len(b) + 1)
    a = list(a)
    while len(a) >= len(b):
        c = f2mul(a[-1], inv)
        k = len(a) - len(b)
        q[k] = c
        for i, y in enumerate(b):
            a[k + i] = f2sub(a[k + i], f2mul(c, y))
        a = ptrim(a[:-1]) if a[-1] == Z2 else ptrim(a)
    return ptrim(q), ptrim(a)


def pmod(a, b):
    return pdivmod(a, b)[1]


def pgcd(a, b):
    a, b = ptrim(a), ptrim(b)
    while b:
        a, b = b, pmod(a, b)
    inv = f2inv(a[-1])
    return [f2mul(x, inv) for x in a]


def ppowmod(base, e, m):
    r, b = [O2], pmod(base, m)
    while e:
        if e & 1:
            r = pmod(pmul(r, b), m)
        b = pmod(pmul(b, b), m)
        e >>= 1
    return r


def interpolate(xs, ys):
    n = len(xs)
    out = [Z2] * n
    for i in range(n):
        num, den = [O2], O2
        for j in range(n):
            if j != i:
                num = pmul(num, [f2sub(Z2, xs[j]), O2])
                den = f2mul(den, f2sub(xs[i], xs[j]))
        c = f2mul(ys[i], f2inv(den))
        for k, v in enumerate(num):
            out[k] = f2add(out[k], f2mul(c, v))
    return ptrim(out)


def roots(p, rng):
    """all roots in Fq2 of p (squarefree part via gcd with t^(q^2) - t)"""
    g = pgcd(p, pmod(f_sub(ppowmod([Z2, O2], Q * Q, p), [Z2, O2]), p))
    out = []
    stack = [g]
    while stack:
        g = stack.pop()
        if len(g) <= 1:
            continue
        if len(g) == 2:
            out.append(f2mul(f2sub(Z2, g[0]), f2inv(g[1])))
            continue
        while True:   # Cantor-Zassenhaus split with a random shift
            c = (rng.randrange(Q), rng.randrange(Q))
            h = ppowmod([c, O2], (Q * Q - 1) // 2, g)
            d = pgcd(g, f_sub(h, [O2]))
            if 1 < len(d) < len(g):
                stack += [d, pdivmod(g, d)[0]]
                break
    return out


def f_sub(a, b):
    n = max(len(a), len(b))
    a = list(a) + [Z2] * (n - len(a))
    b = list(b) + [Z2] * (n - len(b))
    return ptrim([f2sub(x, y) for x, y in zip(a, b)])


# ---- Fq12 helpers ----
def frob2(x):
    return f12pow(x, Q * Q)


def emb6(a):
    """Fq6 -> Fq12 (c0 = a, c1 = 0)"""
    return (a, (Z2, Z2, Z2))


W = ((Z2, Z2, Z2), (O2, Z2, Z2))   # w


def f12add(a, b):
    return tuple(tuple(f2add(x, y) for x, y in zip(p, q)) for p, q in zip(a, b))


def f12sub(a, b):
    return tuple(tuple(f2sub(x, y) for x, y in zip(p, q)) for p, q in zip(a, b))


def f12scal(c, a):
    """c in Fq2 times a"""
    return tuple(tuple(f2mul(c, x) for x in p) for p in a)


def b0(f):
    return f[1][0]


def main():
    rng = random.Random(2026)
    gamma_w = frob2(W)                 # F(w) = gamma w
    for attempt in range(40):
        a0 = tuple((rng.randrange(Q), rng.randrange(Q)) for _ in range(3))
        dl = tuple((rng.randrange(Q), rng.randrange(Q)) for _ in range(3))
        A0, DL = emb6(a0), emb6(dl)
        FA0, FDL = frob2(A0), frob2(DL)

        def parts(t):
            al = f12add(A0, f12scal(t, DL))
            fal = f12add(FA0, f12scal(t, FDL))
            n = f12mul(f12add(al, W), f12add(fal, gamma_w))
            d = f12mul(f12sub(al, W), f12sub(fal, gamma_w))
            return n, d
        ts, ys = [], []
        for k in range(13):
            t = (k + 1, 3 * k + 2)
            n, d = parts(t)
            conj = [d]
            for _ in range(5):
                conj.append(frob2(conj[-1]))
            adj = conj[1]
            for c in conj[2:]:
                adj = f12mul(adj, c)
            ts.append(t)
            ys.append(b0(f12mul(n, adj)))
        P = interpolate(ts, ys)
        if len(P) < 2:
            continue
        for t in roots(P, rng):
            n, d = parts(t)
            f = f12mul(n, f12inv(d))
            if b0(f) != Z2:
                continue
            assert f12mul(f, f12conj(f)) == F12ONE, "not unitary"
            assert f12pow(f, Q ** 4 - Q ** 2 + 1) == F12ONE, "not in G_Phi6"
            assert f[0][2] != Z2, "a2 = 0 too (only the identity has both)"
            out = {"note": "cyclotomic element of Fq12 with b0 = 0 (plain integers, not Montgomery): "
                           "c0 = (a0, a1, a2), c1 = (b0, b1, b2), each Fq2 as [re, im]; made by "
                           "tests/golden/make_karabina_fixture.py",
                   "f": [[[x[0], x[1]] for x in c] for c in f]}
            path = os.path.join(HERE, "karabina_b0zero.json")
            with open(path, "w") as fh:
                json.dump(out, fh, indent=1)
            print("attempt %d: wrote %s" % (attempt, path))
            return
        print("attempt %d: no Fq2 root" % attempt)
    raise SystemExit("no element found")


if __name__ == "__main__":
    main()
