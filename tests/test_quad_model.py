"""CPU model of the quad-cooperative field operations (pairing_amd/csrc/
coop_quad.h, the verifier's quad VM): four 'lanes' per value, lane r holding
limbs 4r..4r+3, with the DPP moves as list permutations -- the same row
sequence as the kernel (CIOS digit broadcast, lowest-limb split, one-lane
shift, three carry rounds).  Checked against Python big integers: the product
must be the unique (T + m q) / 2^392 with m in [0, 2^392) -- the value the
one-lane column-scan leaves return, so the quad VM is bit-identical to the
one-wave VM -- and red must be fl.h red's x - k q, in exact base-2^28 digits.
The GPU test (tests/test_coop_quad.py) compares the kernel itself with the
leaves; this pins the algorithm without a GPU."""
import random

Q = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
M = (1 << 28) - 1
R = 1 << 392
QINV = (-pow(Q, -1, 1 << 28)) % (1 << 28)
KQ = 0x9d835
QL = [(Q >> (28 * i)) & M for i in range(14)] + [0, 0]
U64 = (1 << 64) - 1


def limbs16(v):
    return [(v >> (28 * i)) & M for i in range(13)] + [v >> (28 * 13), 0, 0]


def pieces(l16):
    return [l16[4 * r:4 * r + 4] for r in range(4)]


def value(l16):
    return sum(x << (28 * i) for i, x in enumerate(l16))


def norm(t):
    """t[r][k]: 64-bit lazy accumulators of position 4r + k -> exact digits"""
    o, cy = [], []
    for r in range(4):
        t0, t1, t2, t3 = t[r]
        t1 += t0 >> 28
        t2 += t1 >> 28
        t3 += t2 >> 28
        assert max(t0, t1, t2, t3) <= U64
        o.append([t0 & M, t1 & M, t2 & M, t3 & M])
        cy.append(t3 >> 28)
    for rnd in range(3):
        cin = [0] + cy[:3]                 # quad_perm [3,0,1,2], lane 0 masked
        cy = []
        for r in range(4):
            v = o[r][0] + cin[r]
            o[r][0] = v & M
            k = v >> 28
            for j in range(1, 4):
                o[r][j] += k
                k = o[r][j] >> 28
                o[r][j] &= M
            cy.append(k)
    return [x for r in range(4) for x in o[r]]


def mont(a16, b16, c16=None, d16=None):
    """a (whole) * b (pieces) [+ c * d] R'^-1 as the quad computes it"""
    bp, dp = pieces(b16), pieces(d16) if d16 else None
    qp = pieces(QL)
    t = [[0, 0, 0, 0] for _ in range(4)]
    for i in range(14):
        for r in range(4):
            for k in range(4):
                t[r][k] += a16[i] * bp[r][k] + (c16[i] * dp[r][k] if c16 else 0)
        m = ((t[0][0] & 0xffffffff) * QINV) & M        # lane 0, broadcast (quad_perm [0,0,0,0])
        lo = []
        for r in range(4):
            for k in range(4):
                t[r][k] += m * qp[r][k]
                assert t[r][k] <= U64, "accumulator overflow"
            lo.append(t[r][0] & M)
        assert lo[0] == 0                              # the dropped limb
        nx = lo[1:] + [lo[0]]                          # quad_perm [1,2,3,0]
        for r in range(4):
            t[r][1] += t[r][0] >> 28
            t[r] = [t[r][1], t[r][2], t[r][3], nx[r]]
    return norm(t)


def red(x16):
    x12, x13 = x16[12], x16[13]
    k = ((x13 * KQ + ((x12 * KQ) >> 28)) >> 36) & 0xffffffff
    v = [x16[i] - k * QL[i] for i in range(16)]
    o, cy = [], []
    for r in range(4):
        w = v[4 * r:4 * r + 4]
        for j in range(1, 4):
            w[j] += w[j - 1] >> 28
        o.append([x & M for x in w])
        cy.append(w[3] >> 28)
    for rnd in range(3):
        cin = [0] + cy[:3]
        cy = []
        for r in range(4):
            w = o[r][0] + cin[r]
            o[r][0] = w & M
            for j in range(1, 4):
                w = o[r][j] + (w >> 28)
                o[r][j] = w & M
            cy.append(w >> 28)
    return [x for r in range(4) for x in o[r]]


def lazy(g, u, edge=None):
    out = [0] * 16
    for _ in range(u):
        v = {"max": 2 * Q - 1, "zero": 0}.get(edge, g.randrange(2 * Q))
        for i, d in enumerate(limbs16(v)):
            out[i] += d
    return out


def expected_product(t):
    m = (-t * pow(Q, -1, R)) % R
    return limbs16((t + m * Q) // R)


def test_quad_mont_model_matches_unique_montgomery_digits():
    g = random.Random(5)
    for ua, ub in [(1, 1), (4, 4), (16, 1), (1, 16), (2, 8)]:
        for t in range(60):
            edge = "max" if t == 0 else "zero" if t == 1 else None
            a, b = lazy(g, ua, edge), lazy(g, ub)
            got = mont(a, b)
            assert got == expected_product(value(a) * value(b))
            assert value(got) < 2 * Q


def test_quad_sop2_model():
    g = random.Random(6)
    for (ua, ub), (uc, ud) in [((4, 2), (3, 3)), ((8, 2), (1, 1)), ((1, 1), (16, 1))]:
        for t in range(40):
            edge = "max" if t == 0 else None
            a, b, c, d = lazy(g, ua, edge), lazy(g, ub, edge), lazy(g, uc), lazy(g, ud, edge)
            assert mont(a, b, c, d) == expected_product(value(a) * value(b) + value(c) * value(d))


def test_quad_red_model_matches_fl_red():
    g = random.Random(7)
    for u in (1, 4, 16):
        for t in range(60):
            edge = "max" if t == 0 else "zero" if t == 1 else None
            x = lazy(g, u, edge)
            v = value(x)
            k = ((x[13] * KQ + ((x[12] * KQ) >> 28)) >> 36) & 0xffffffff
            got = red(x)
            assert got == limbs16(v - k * Q)
            assert value(got) % Q == v % Q and value(got) < 2 * Q
