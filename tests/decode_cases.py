"""Encoded-point test cases: the reference's invalid-vector suites
(src/bls12_381/tests/mod.rs:98-560, test_g{1,2}_{uncompressed,compressed}_invalid_vectors)
re-expressed as (record bytes, expected GroupDecodingError status), plus
random garbage and on-curve-but-not-in-subgroup points.  Pure Python ints
(canonical values) -- independent of the oracle and of the product.

Status codes (include/pairing_amd.h PA_DECODE_*): 0 Ok, 1 NotOnCurve,
2 NotInSubgroup, 3 x/x.c0, 4 x.c1, 5 y/y.c0, 6 y.c1 (CoordinateDecodingError),
7 UnexpectedCompressionMode, 8 UnexpectedInformation.
"""
import numpy as np

from helpers import Q
from pymodel import f2add, f2mul

OK, NOT_ON_CURVE, NOT_IN_SUBGROUP = 0, 1, 2
X_C0, X_C1, Y_C0, Y_C1 = 3, 4, 5, 6
COMPRESSION_MODE, INFORMATION = 7, 8

G1_X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1_Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1
G2_X = (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E)
G2_Y = (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE)
B1 = 4
B2 = (4, 4)
QM1_2 = (Q - 1) // 2


def be(v):
    return v.to_bytes(48, "big")


def is_square_fq(a):
    return a % Q == 0 or pow(a, QM1_2, Q) == 1


def sqrt_fq(a):
    return pow(a, (Q + 1) // 4, Q)


def f2pow(a, e):
    r = (1, 0)
    for bit in bin(e)[2:]:
        r = f2mul(r, r)
        if bit == "1":
            r = f2mul(r, a)
    return r


def is_square_fq2(a):
    return is_square_fq(a[0] * a[0] + a[1] * a[1])


def sqrt_fq2(a):
    """Algorithm 9 of eprint 2012/685 (the one fq2.rs:167-220 follows)"""
    if a == (0, 0):
        return (0, 0)
    a1 = f2pow(a, (Q - 3) // 4)
    alpha = f2mul(f2mul(a1, a1), a)
    x0 = f2mul(a1, a)
    if alpha == (Q - 1, 0):
        return f2mul(x0, (0, 1))
    b = f2pow(f2add(alpha, (1, 0)), (Q - 1) // 2)
    return f2mul(b, x0)


def rhs1(x):
    return (x * x * x + B1) % Q


def rhs2(x):
    return f2add(f2mul(f2mul(x, x), x), B2)


def enc_g1(x, y, compressed, greatest=False):
    if compressed:
        b = bytearray(be(x))
        b[0] |= 0x80 | (0x20 if greatest else 0)
        return bytes(b)
    return be(x) + be(y)


def enc_g2(x, y, compressed, greatest=False):
    if compressed:
        b = bytearray(be(x[1]) + be(x[0]))
        b[0] |= 0x80 | (0x20 if greatest else 0)
        return bytes(b)
    return be(x[1]) + be(x[0]) + be(y[1]) + be(y[0])


def zero_enc(size, compressed):
    b = bytearray(size)
    b[0] = 0x40 | (0x80 if compressed else 0)
    return bytes(b)


def _infinity_cases(size, compressed):
    """the `z` blocks of the reference suites"""
    z = zero_enc(size, compressed)
    out = [(z, OK)]
    t = bytearray(z)
    if compressed:
        t[0] &= 0x7F
    else:
        t[0] |= 0x80
    out.append((bytes(t), COMPRESSION_MODE))
    t = bytearray(z)
    t[0] |= 0x20
    out.append((bytes(t), INFORMATION))
    for i in range(size):
        t = bytearray(z)
        t[i] |= 0x01
        out.append((bytes(t), INFORMATION))
    return out


def _with(rec, offset, chunk, set_flags=0):
    b = bytearray(rec)
    b[offset:offset + len(chunk)] = chunk
    b[0] |= set_flags
    return bytes(b)


def g1_cases(compressed):
    size = 48 if compressed else 96
    out = _infinity_cases(size, compressed)
    o = enc_g1(G1_X, G1_Y, compressed)
    out.append((o, OK))
    t = bytearray(o)
    if compressed:
        t[0] &= 0x7F
    else:
        t[0] |= 0x80
    out.append((bytes(t), COMPRESSION_MODE))
    fl = 0x80 if compressed else 0
    out.append((_with(o, 0, be(Q), fl), X_C0))
    if not compressed:
        out.append((_with(o, 48, be(Q)), Y_C0))
        out.append((_with(o, 0, be(0)), NOT_ON_CURVE))
        out.append((_with(o, 0, be(G1_X), 0x20), INFORMATION))
        x = 1
        while not is_square_fq(rhs1(x)):
            x += 1
        out.append((enc_g1(x, sqrt_fq(rhs1(x)), False), NOT_IN_SUBGROUP))
    else:
        x = 1         # the first x with no point on the curve
        while is_square_fq(rhs1(x)):
            x += 1
        out.append((enc_g1(x, None, True), NOT_ON_CURVE))
        x = 1
        while not is_square_fq(rhs1(x)):
            x += 1
        out.append((enc_g1(x, None, True), NOT_IN_SUBGROUP))
        out.append((enc_g1(x, None, True, greatest=True), NOT_IN_SUBGROUP))
    return out


def g2_cases(compressed):
    size = 96 if compressed else 192
    out = _infinity_cases(size, compressed)
    o = enc_g2(G2_X, G2_Y, compressed)
    out.append((o, OK))
    t = bytearray(o)
    if compressed:
        t[0] &= 0x7F
    else:
        t[0] |= 0x80
    out.append((bytes(t), COMPRESSION_MODE))
    fl = 0x80 if compressed else 0
    out.append((_with(o, 0, be(Q), fl), X_C1))
    out.append((_with(o, 48, be(Q), fl), X_C0))
    if not compressed:
        out.append((_with(o, 96, be(Q)), Y_C1))
        out.append((_with(o, 144, be(Q)), Y_C0))
        out.append((_with(_with(o, 0, be(0)), 48, be(0)), NOT_ON_CURVE))
        x = (1, 0)
        while not is_square_fq2(rhs2(x)):
            x = f2add(x, (1, 0))
        out.append((enc_g2(x, sqrt_fq2(rhs2(x)), False), NOT_IN_SUBGROUP))
    else:
        x = (1, 1)
        while is_square_fq2(rhs2(x)):
            x = f2add(x, (1, 0))
        out.append((enc_g2(x, None, True), NOT_ON_CURVE))
        x = (1, 1)
        while not is_square_fq2(rhs2(x)):
            x = f2add(x, (1, 0))
        out.append((enc_g2(x, None, True), NOT_IN_SUBGROUP))
        out.append((enc_g2(x, None, True, greatest=True), NOT_IN_SUBGROUP))
    return out


def garbage(gen, n, size, compressed):
    """random records with the mode bit right and the infinity bit clear:
    mostly CoordinateDecodingError / NotOnCurve, a few valid-looking x"""
    b = gen.integers(0, 256, size=(n, size), dtype=np.uint8)
    # half the records with every coordinate below q so the curve checks run
    for off in range(0, size, 48):
        b[0::2, off] &= 0x0F
    b[:, 0] &= 0x1F if not compressed else 0x3F
    if compressed:
        b[:, 0] |= 0x80
    return b


def as_array(cases, size):
    enc = np.frombuffer(b"".join(c[0] for c in cases), np.uint8).reshape(-1, size)
    want = np.array([c[1] for c in cases], np.uint8)
    return enc.copy(), want


# ---------------- subgroup-membership cases ----------------
# On-curve points in and out of the prime-order subgroups, including points
# with small-order components, to pin the GPU's endomorphism membership test
# (kernels_decode.hip in_subgroup) to the reference's r * P == 0
# (ec.rs:142-144) as evaluated by the oracle.  Affine Python-int arithmetic.
R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
_X = -0xd201000000010000
H1 = 0x396c8c005555e1568c00aaab0000aaab
H2 = (_X ** 8 - 4 * _X ** 7 + 5 * _X ** 6 - 4 * _X ** 4 + 6 * _X ** 3 - 4 * _X ** 2 - 4 * _X + 13) // 9


def _f1():
    inv = lambda a: pow(a, -1, Q)
    return dict(add=lambda a, b: (a + b) % Q, sub=lambda a, b: (a - b) % Q, mul=lambda a, b: a * b % Q,
                inv=inv, zero=0, small=lambda k: k % Q)


def _f2():
    from pymodel import f2inv, f2sub
    return dict(add=f2add, sub=f2sub, mul=f2mul, inv=f2inv, zero=(0, 0), small=lambda k: (k % Q, 0))


def _ec_add(F, P, R):
    if P is None:
        return R
    if R is None:
        return P
    (x1, y1), (x2, y2) = P, R
    if x1 == x2:
        if F["add"](y1, y2) == F["zero"]:
            return None
        lam = F["mul"](F["mul"](F["small"](3), F["mul"](x1, x1)), F["inv"](F["add"](y1, y1)))
    else:
        lam = F["mul"](F["sub"](y2, y1), F["inv"](F["sub"](x2, x1)))
    x3 = F["sub"](F["sub"](F["mul"](lam, lam), x1), x2)
    return (x3, F["sub"](F["mul"](lam, F["sub"](x1, x3)), y1))


def _ec_mul(F, P, k):
    acc = None
    for bit in bin(k)[2:]:
        acc = _ec_add(F, acc, acc)
        if bit == "1":
            acc = _ec_add(F, acc, P)
    return acc


def _random_point(group, g):
    while True:
        if group == 1:
            x = int(g.integers(0, 1 << 62)) * (1 << 300) % Q + int(g.integers(0, 1 << 62))
            if is_square_fq(rhs1(x)):
                return (x, sqrt_fq(rhs1(x)))
        else:
            x = (int(g.integers(0, 1 << 62)) << 200, int(g.integers(0, 1 << 62)) + 7)
            if is_square_fq2(rhs2(x)):
                return (x, sqrt_fq2(rhs2(x)))


def subgroup_points(group, seed, n=6):
    """(points, in_subgroup) for uncompressed encoding: random curve points,
    their cofactor-cleared and r-multiplied images (small-order only), order-3
    and order-13 (G2) torsion points, and sums of subgroup and torsion points."""
    F = _f1() if group == 1 else _f2()
    h = H1 if group == 1 else H2
    small = 3 if group == 1 else 13
    g = np.random.default_rng(seed)
    pts = []
    for _ in range(n):
        R = _random_point(group, g)
        S = _ec_mul(F, R, h)             # in the subgroup
        T = _ec_mul(F, R, R_ORDER)       # order divides h: outside
        Ts = _ec_mul(F, T, h // small)   # order `small` or trivial
        pts += [R, S, T, _ec_add(F, S, T)]
        if Ts is not None:
            pts += [Ts, _ec_add(F, S, Ts)]
    pts = [P for P in pts if P is not None]
    truth = [_ec_mul(F, P, R_ORDER) is None for P in pts]
    return pts, truth


def aff_record(group, P):
    """the ABI affine record (pa_g1_affine 13 / pa_g2_affine 25 u64, Montgomery
    coordinates, infinity word last) of a point P = (x, y), or of None (infinity)"""
    from helpers import mont
    w = 13 if group == 1 else 25
    if P is None:
        r = [0] * w
        r[-1] = 1
        return r
    x, y = P
    if group == 1:
        return mont(x) + mont(y) + [0]
    return mont(x[0]) + mont(x[1]) + mont(y[0]) + mont(y[1]) + [0]


def subgroup_records(group, seed, n=6):
    pts, truth = subgroup_points(group, seed, n)
    enc = enc_g1 if group == 1 else enc_g2
    recs = [enc(P[0], P[1], False) for P in pts]
    size = 96 if group == 1 else 192
    return np.frombuffer(b"".join(recs), np.uint8).reshape(-1, size).copy(), np.array(truth)
