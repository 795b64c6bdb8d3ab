"""An independent pure-Python model of the BLS12-381 tower over canonical
integers (no Montgomery form, no limbs), used only by the CPU tests to
cross-check the C oracle on small cases.  Written from the tower definition
(src/bls12_381/README.md: u^2 = -1, v^3 = u + 1, w^2 = v), not from the
reference's formulas, so it shares no code path with oracle/ or pairing_amd/.

Element encodings: Fq = int; Fq2 = (c0, c1); Fq6 = (Fq2, Fq2, Fq2);
Fq12 = (Fq6, Fq6).  `to_limbs`/`from_limbs` convert to/from the 72-word
Montgomery ABI layout.
"""
from helpers import Q, limbs, mont, unmont

# ---- Fq2 ----
def f2add(a, b): return ((a[0] + b[0]) % Q, (a[1] + b[1]) % Q)
def f2sub(a, b): return ((a[0] - b[0]) % Q, (a[1] - b[1]) % Q)
def f2neg(a): return ((-a[0]) % Q, (-a[1]) % Q)
def f2mul(a, b): return ((a[0] * b[0] - a[1] * b[1]) % Q, (a[0] * b[1] + a[1] * b[0]) % Q)
def f2xi(a): return ((a[0] - a[1]) % Q, (a[0] + a[1]) % Q)  # * (u + 1)
def f2inv(a):
    n = (a[0] * a[0] + a[1] * a[1]) % Q
    ni = pow(n, Q - 2, Q)
    return (a[0] * ni % Q, (-a[1]) * ni % Q)

F2ZERO, F2ONE = (0, 0), (1, 0)

# ---- Fq6 = Fq2[v]/(v^3 - xi): schoolbook ----
def f6add(a, b): return tuple(f2add(x, y) for x, y in zip(a, b))
def f6sub(a, b): return tuple(f2sub(x, y) for x, y in zip(a, b))
def f6neg(a): return tuple(f2neg(x) for x in a)
def f6mul(a, b):
    c = [F2ZERO] * 5
    for i in range(3):
        for j in range(3):
            c[i + j] = f2add(c[i + j], f2mul(a[i], b[j]))
    return (f2add(c[0], f2xi(c[3])), f2add(c[1], f2xi(c[4])), c[2])
def f6v(a): return (f2xi(a[2]), a[0], a[1])  # * v

F6ZERO = (F2ZERO, F2ZERO, F2ZERO)
F6ONE = (F2ONE, F2ZERO, F2ZERO)

# ---- Fq12 = Fq6[w]/(w^2 - v): schoolbook ----
def f12mul(a, b):
    c0 = f6add(f6mul(a[0], b[0]), f6v(f6mul(a[1], b[1])))
    c1 = f6add(f6mul(a[0], b[1]), f6mul(a[1], b[0]))
    return (c0, c1)
def f12sqr(a): return f12mul(a, a)
def f12conj(a): return (a[0], f6neg(a[1]))

F12ONE = (F6ONE, F6ZERO)


def f12pow(a, e):
    r = F12ONE
    base = a
    while e:
        if e & 1:
            r = f12mul(r, base)
        base = f12sqr(base)
        e >>= 1
    return r


def f12inv(a):
    # a^(q^12 - 2) is too slow; use the norm to Fq6: (a0 + a1 w)(a0 - a1 w) = a0^2 - v a1^2
    n = f6sub(f6mul(a[0], a[0]), f6v(f6mul(a[1], a[1])))
    ni = f6inv(n)
    return (f6mul(a[0], ni), f6neg(f6mul(a[1], ni)))


def f6inv(a):
    # via the Fq2-linear norm: solve with the adjugate of the multiplication matrix
    c0 = f2sub(f2mul(a[0], a[0]), f2xi(f2mul(a[1], a[2])))
    c1 = f2sub(f2xi(f2mul(a[2], a[2])), f2mul(a[0], a[1]))
    c2 = f2sub(f2mul(a[1], a[1]), f2mul(a[0], a[2]))
    t = f2add(f2mul(a[0], c0), f2xi(f2add(f2mul(a[2], c1), f2mul(a[1], c2))))
    ti = f2inv(t)
    return (f2mul(c0, ti), f2mul(c1, ti), f2mul(c2, ti))


# ---- conversions to the 72-word Montgomery ABI layout ----
def fq12_to_limbs(a):
    out = []
    for f6 in a:
        for f2 in f6:
            for x in f2:
                out += mont(x)
    return out


def fq12_from_limbs(ws):
    ws = [int(w) for w in ws]
    vals = [unmont(ws[6 * k:6 * k + 6]) for k in range(12)]
    f2s = [(vals[2 * k], vals[2 * k + 1]) for k in range(6)]
    return ((f2s[0], f2s[1], f2s[2]), (f2s[3], f2s[4], f2s[5]))


def fq2_from_limbs(ws):
    ws = [int(w) for w in ws]
    return (unmont(ws[:6]), unmont(ws[6:12]))


__all__ = [n for n in dir() if not n.startswith("_")] + ["limbs"]
