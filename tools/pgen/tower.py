"""BLS12-381 tower, line functions, Miller loop and final exponentiation
written against the tracing DSL (dsl.py).  The formulas are those of
pairing_amd/csrc/tower_fl.h / pairing_fl.h (themselves the reference's:
fq2.rs, fq6.rs, fq12.rs, mod.rs -- cited per function below); the bound of
every value is tracked by the DSL, and red() is placed exactly where the
next operation's bound check needs it.

Element encodings: Fq2 = (c0, c1) of Val; Fq6 = 3-tuple of Fq2;
Fq12 = (Fq6, Fq6).
"""
import os

from dsl import SUBCU, Q

X_ABS = 0xD201000000010000  # |x|, x < 0 (mod.rs:23-25)


def _frob_consts():
    """Frobenius coefficients (fq.rs:139-498) as field values, derived as in
    tools/gen_consts.py."""
    import gen_consts as g
    return g.FROB_FQ6_C1, g.FROB_FQ6_C2, g.FROB_FQ12_C1


class NormStop(Exception):
    """raised by inv2 in a norm-only program (Tower.fe_split == "norm"):
    args[0] is the Fq value the base-field inversion would invert"""


KSQR_LAZY_XI = __import__("os").environ.get("PGEN_KSQR_LAZY_XI", "1") == "1"


class Tower:
    # split final exponentiation (kernels.final_exp_prog(split=...)): "norm"
    # stops at the base-field value to invert (NormStop), "inv" reads its
    # inverse from input slot 12 instead of running the Fermat chain
    fe_split = None

    def __init__(self, p):
        self.p = p

    # ---------------- Fq2 ----------------
    def add2(self, a, b): return (self.p.add(a[0], b[0]), self.p.add(a[1], b[1]))
    def sub2(self, a, b): return (self.p.sub(a[0], b[0]), self.p.sub(a[1], b[1]))
    def neg2(self, a): return (self.p.neg(a[0]), self.p.neg(a[1]))
    def dbl2(self, a): return self.add2(a, a)
    def red2(self, a): return (self.p.red(a[0]), self.p.red(a[1]))
    def u2(self, a): return max(a[0].u, a[1].u)

    def nu(self, x):
        """limb bound of neg(x) (dsl.Prog.sub_key / sub_bounds)"""
        return self.p.neg_u(x)

    def xi(self, a):  # fq2.rs:41-45, * (u + 1)
        return (self.p.sub(a[0], a[1]), self.p.add(a[0], a[1]))

    def conj2(self, a):
        return (a[0], self.p.neg(a[1]))

    def mul2(self, a, b):  # fq2.rs:123-136, schoolbook, one reduction per coordinate
        p = self.p
        if self.nu(a[1]) * b[1].u <= a[1].u * self.nu(b[1]):
            c0 = p.sop(a[0], b[0], p.neg(a[1]), b[1])
        else:
            c0 = p.sop(a[0], b[0], a[1], p.neg(b[1]))
        c1 = p.sop(a[0], b[1], a[1], b[0])
        return (c0, c1)

    def sqr2(self, a):  # fq2.rs:87-101
        p = self.p
        if (a[0].u + a[1].u) * (a[0].u + self.nu(a[1])) <= 17:
            c0 = p.mul(p.add(a[0], a[1]), p.sub(a[0], a[1]))
        else:
            c0 = p.sop(a[0], a[0], p.neg(a[1]), a[1])
        c1 = p.mul(p.dbl(a[0]), a[1])
        return (c0, c1)

    def mul_fq(self, a, b):
        return (self.p.mul(a[0], b), self.p.mul(a[1], b))

    def lim2(self, a):
        return a if self.u2(a) <= 2 else self.red2(a)

    def const2(self, c):
        return (self.p.const(c[0]), self.p.const(c[1]))

    def one2(self):
        return (self.p.const(1), self.p.const(0))

    # ---------------- Fq6 ----------------
    def add6(self, a, b): return tuple(self.add2(x, y) for x, y in zip(a, b))
    def sub6(self, a, b): return tuple(self.sub2(x, y) for x, y in zip(a, b))
    def neg6(self, a): return tuple(self.neg2(x) for x in a)
    def red6(self, a): return tuple(self.red2(x) for x in a)
    def u6(self, a): return max(self.u2(x) for x in a)
    def mul_v(self, a): return (self.xi(a[2]), a[0], a[1])  # fq6.rs:32-38

    def mul6(self, a, b):  # fq6.rs:199-248, Karatsuba
        assert self.u6(a) <= 2 and self.u6(b) <= 2
        t = self
        v0 = t.mul2(a[0], b[0])
        v1 = t.mul2(a[1], b[1])
        v2 = t.mul2(a[2], b[2])
        t0 = t.mul2(t.lim2(t.add2(a[1], a[2])), t.lim2(t.add2(b[1], b[2])))
        t1 = t.mul2(t.lim2(t.add2(a[0], a[1])), t.lim2(t.add2(b[0], b[1])))
        t2 = t.mul2(t.lim2(t.add2(a[0], a[2])), t.lim2(t.add2(b[0], b[2])))
        c0 = t.red2(t.add2(t.xi(t.sub2(t0, t.add2(v1, v2))), v0))
        c1 = t.red2(t.add2(t.sub2(t1, t.add2(v0, v1)), t.xi(v2)))
        c2 = t.red2(t.add2(t.sub2(t2, t.add2(v0, v2)), v1))
        return (c0, c1, c2)

    def mul_by_1(self, a, c1):  # fq6.rs:40-66
        xc = self.xi(c1)
        return (self.mul2(a[2], xc), self.mul2(a[0], c1), self.mul2(a[1], c1))

    def mul_by_01(self, a, c0, c1):  # fq6.rs:68-109
        t = self
        a_a = t.mul2(a[0], c0)
        b_b = t.mul2(a[1], c1)
        t1 = t.mul2(c1, t.lim2(t.add2(a[1], a[2])))
        t3 = t.mul2(c0, t.lim2(t.add2(a[0], a[2])))
        t2 = t.mul2(t.lim2(t.add2(c0, c1)), t.lim2(t.add2(a[0], a[1])))
        r0 = t.red2(t.add2(t.xi(t.sub2(t1, b_b)), a_a))
        r1 = t.red2(t.sub2(t2, t.add2(a_a, b_b)))
        r2 = t.red2(t.add2(t.sub2(t3, a_a), b_b))
        return (r0, r1, r2)

    def frob6(self, a, power):  # fq6.rs:157-164
        c6_1, c6_2, _ = _frob_consts()
        if power & 1:
            a = tuple(self.red2(self.conj2(x)) for x in a)
        return (a[0], self.mul2(a[1], self.const2(c6_1[power % 6])),
                self.mul2(a[2], self.const2(c6_2[power % 6])))

    # ---------------- Fq12 ----------------
    def conj12(self, a):  # fq12.rs:30-32
        return (a[0], self.red6(self.neg6(a[1])))

    # Operation order matters for register pressure (the allocator follows
    # it): the product with freshly computed operands goes first, while the
    # plain operands (often variable-backed, free to drop and re-read) wait.
    def mul12(self, a, b):  # fq12.rs:116-130
        t = self
        cross = t.mul6(t.add6(a[0], a[1]), t.add6(b[0], b[1]))
        aa = t.mul6(a[0], b[0])
        bb = t.mul6(a[1], b[1])
        c1 = t.red6(t.sub6(cross, t.add6(aa, bb)))
        c0 = t.red6(t.add6(t.mul_v(bb), aa))
        return (c0, c1)

    def sqr12(self, a):  # fq12.rs:99-114
        t = self
        s = t.mul6(t.red6(t.add6(t.mul_v(a[1]), a[0])), t.add6(a[0], a[1]))
        ab = t.mul6(a[0], a[1])
        c0 = t.red6(t.sub6(s, t.add6(ab, t.mul_v(ab))))
        c1 = t.red6(t.add6(ab, ab))
        return (c0, c1)

    def mul_by_014(self, a, c0, c1, c4):  # fq12.rs:34-48
        t = self
        s = t.mul_by_01(t.red6(t.add6(a[1], a[0])), c0, t.lim2(t.add2(c1, c4)))
        aa = t.mul_by_01(a[0], c0, c1)
        bb = t.mul_by_1(a[1], c4)
        r1 = t.red6(t.sub6(s, t.add6(aa, bb)))
        r0 = t.red6(t.add6(t.mul_v(bb), aa))
        return (r0, r1)

    def frob12(self, a, power):  # fq12.rs:90-97
        _, _, c12 = _frob_consts()
        c0 = self.frob6(a[0], power)
        c1 = self.frob6(a[1], power)
        k = self.const2(c12[power % 12])
        return (c0, tuple(self.mul2(x, k) for x in c1))

    def fq4_sqr(self, a, b):
        t = self
        t0 = t.sqr2(a)
        t1 = t.sqr2(b)
        t2 = t.sqr2(t.add2(a, b))
        r1 = t.red2(t.sub2(t2, t.add2(t0, t1)))
        r0 = t.red2(t.add2(t.xi(t1), t0))
        return r0, r1

    def cyc_sqr(self, f):
        """Granger-Scott squaring (value of Fq12::square on the cyclotomic subgroup)"""
        t = self
        (a0, a1, a2), (b0, b1, b2) = f
        # one Fq4 pair at a time: its two outputs are finished before the next
        # pair's squarings, so at most one pair of temporaries is live
        t0, t1 = t.fq4_sqr(a0, b1)
        c00 = t.red2(t.add2(t.dbl2(t.sub2(t0, a0)), t0))
        c11 = t.red2(t.add2(t.dbl2(t.add2(t1, b1)), t1))
        t2, t3 = t.fq4_sqr(b0, a2)
        t4, t5 = t.fq4_sqr(a1, b2)
        t5x = t.xi(t5)
        c10 = t.red2(t.add2(t.dbl2(t.add2(t5x, b0)), t5x))
        c01 = t.red2(t.add2(t.dbl2(t.sub2(t2, a1)), t2))
        c12 = t.red2(t.add2(t.dbl2(t.add2(t3, b2)), t3))
        c02 = t.red2(t.add2(t.dbl2(t.sub2(t4, a2)), t4))
        return ((c00, c01, c02), (c10, c11, c12))

    # ---------------- compressed cyclotomic squaring (Karabina) ----------------
    # f = (a0 + a1 v + a2 v^2) + (b0 + b1 v + b2 v^2) w in the cyclotomic subgroup
    # is determined by g = (a1, a2, b0, b2) (S. Karabina, "Squaring in cyclotomic
    # subgroups", eprint 2010/542; the formulas of Aranha-Karabina-Longa-Gebotys-
    # Lopez, eprint 2010/526, section 5, in this tower's coordinates).  Squaring
    # g costs 6 Fq2 squarings against Granger-Scott's 9 on all of f; recovering
    # a0, b1 costs one Fq2 division, so a run of squarings stays compressed and
    # only the powers that are multiplied are decompressed, their divisions
    # sharing one inversion (Montgomery's trick).  Checked against the Python
    # model in tests/test_pgen.py (test_karabina_*).
    def ksqr(self, g):
        """g -> g^2 compressed:  a1' = 3(b0^2 + xi a2^2) - 2 a1,
        a2' = 3(a1^2 + xi b2^2) - 2 a2,  b0' = 6 xi a1 b2 + 2 b0,  b2' = 6 a2 b0 + 2 b2"""
        t = self
        a1, a2, b0, b2 = g

        def half(x, y, z, zy, xi_on_cross):
            # x^2 + xi y^2 and 2 x y = (x + y)^2 - x^2 - y^2, then
            # z' = 3 (x^2 + xi y^2) - 2 z  and  zy' = 6 [xi] x y + 2 zy
            sx, sy = t.sqr2(x), t.sqr2(y)
            sxy = t.sqr2(t.lim2(t.add2(x, y)))
            s = t.red2(t.add2(sx, t.xi(sy)))
            c = t.red2(t.sub2(sxy, t.add2(sx, sy)))
            if xi_on_cross:
                # carry-normalized programs leave xi(c) as it is: 3 c + 2 zy below
                # is reduced anyway, and its bounds hold (checked by dsl.evaluate)
                c = t.xi(c) if t.p.use_norm and KSQR_LAZY_XI else t.red2(t.xi(c))
            nz = t.red2(t.add2(t.dbl2(t.sub2(s, z)), s))
            nzy = t.red2(t.add2(t.dbl2(t.add2(c, zy)), c))
            return nz, nzy

        na2, nb0 = half(a1, b2, a2, b0, True)
        na1, nb2 = half(b0, a2, a1, b2, False)
        return (na1, na2, nb0, nb2)

    def kdec_numden(self, g):
        """the division that recovers b1 = num / den:  b0 != 0: (3 a1^2 - 2 a2 +
        xi b2^2) / (4 b0);  b0 == 0: 2 a1 b2 / a2 (lane-wise select).  Only the
        identity has b0 = a2 = 0 (then num = den = 0, and the shared inversion's
        0 -> 0 gives b1 = 0, a0 = 1: the identity).  Also returns
        w = 3 a1 a2 - b0 b2 (a0 = xi (2 b1^2 - w) + 1), formed now so that the
        finish does not read g again."""
        t, p = self, self.p
        a1, a2, b0, b2 = g
        s1 = t.sqr2(a1)
        num1 = t.red2(t.sub2(t.add2(t.add2(t.dbl2(s1), s1), t.xi(t.sqr2(b2))), t.dbl2(a2)))
        den1 = t.red2(t.dbl2(t.dbl2(b0)))
        num2 = t.red2(t.dbl2(t.mul2(a1, b2)))
        den2 = t.red2(a2)
        z = [p.red_full(b0[0]), p.red_full(b0[1])]
        num = (p.selz(z, num2[0], num1[0]), p.selz(z, num2[1], num1[1]))
        den = (p.selz(z, den2[0], den1[0]), p.selz(z, den2[1], den1[1]))
        # w = 3 a1 a2 - b0 b2 as two 4-term products:
        #   re = 3 a1r a2r + 3 (-a1i) a2i + (-b0r) b2r + b0i b2i
        #   im = 3 a1r a2i + 3 a1i a2r + (-b0r) b2i + (-b0i) b2r
        a13 = (t.lim2(t.add2(t.dbl2(a1), a1)))
        nb0 = (p.neg(b0[0]), p.neg(b0[1]))
        w = (p.sopn([a13[0], a2[0], p.neg(a13[1]), a2[1], nb0[0], b2[0], b0[1], b2[1]]),
             p.sopn([a13[0], a2[1], a13[1], a2[0], nb0[0], b2[1], nb0[1], b2[0]]))
        return num, den, w

    def kdec_finish(self, g, num, iden, w):
        """b1 = num iden, a0 = xi (2 b1^2 - w) + 1"""
        t = self
        a1, a2, b0, b2 = g
        b1 = t.mul2(num, iden)
        s = t.red2(t.sub2(t.dbl2(t.sqr2(b1)), w))
        a0 = t.red2(t.add2(t.xi(s), t.one2()))
        return ((a0, a1, a2), (b0, b1, b2))

    def inv2_direct(self, a, tag):
        """Fq2 inverse (fq2.rs:138-155) with the base-field inversion as one op"""
        p = self.p
        n = p.sop(a[0], a[0], a[1], a[1])
        i = self.inv_fq(n, tag)
        return (p.mul(a[0], i), p.mul(p.neg(a[1]), i))

    def batch_inv2(self, ds, tag):
        """Montgomery's trick over Fq2 values: 3 (n - 1) products + one inverse"""
        t = self
        pre = [ds[0]]
        for d in ds[1:]:
            pre.append(t.mul2(pre[-1], d))
        acc = t.inv2_direct(pre[-1], tag)
        out = [None] * len(ds)
        for k in range(len(ds) - 1, 0, -1):
            out[k] = t.mul2(acc, pre[k - 1])
            acc = t.mul2(acc, ds[k])
        out[0] = acc
        return out

    # ---------------- inversion ----------------
    def inv_fq(self, a, tag):
        """a^(q-2) (Fermat; the same value as fq.rs:849-902's Euclid for a != 0):
        a sliding window of 4 bits over the constant exponent -- 8 odd powers,
        then 380 squarings and 78 multiplications (463 products against 608 for
        bitwise square-and-multiply); PGEN_INV_W=0 selects the bitwise form.
        One-lane programs with binary GCD (Prog.binv_ok): the in-kernel binary
        GCD instead (~37 k instructions against ~300 k)."""
        if getattr(self.p, "binv_ok", False):
            return self.p.binv(self.p.red_full(a))
        W = int(os.environ.get("PGEN_INV_W", "4"))
        if W:
            return self._inv_fq_window(a, tag, W)
        p = self.p
        e = Q - 2
        assert e.bit_length() == 381
        va, vr = "inv_a_" + tag, "inv_r_" + tag
        p.var(va)
        p.var(vr)
        p.set(va, a)
        p.set(vr, a)  # top bit (380)
        # bits 379..0 in words: [379..320] then five 64-bit words
        spans = [(320, 60)] + [(64 * w, 64) for w in range(4, -1, -1)]
        for lo, nbits in spans:
            mask = (e >> lo) & ((1 << nbits) - 1)
            with p.loop(nbits) as L:
                p.set(vr, p.sqr(p.get(vr)))
                with p.if_bit(mask, L):
                    p.set(vr, p.mul(p.get(vr), p.get(va)))
        return p.get(vr)

    def _inv_fq_window(self, a, tag, W):
        p = self.p
        bits = bin(Q - 2)[2:]
        wins, i, zeros = [], 0, 0          # (squarings before the window's multiply, odd value)
        while i < len(bits):
            if bits[i] == "0":
                zeros += 1
                i += 1
                continue
            j = min(i + W, len(bits))
            while bits[j - 1] == "0":
                j -= 1
            wins.append((zeros + (j - i), int(bits[i:j], 2)))
            zeros, i = 0, j
        tail = zeros
        names = ["inv_t%d_%s" % (k, tag) for k in range(1 << (W - 1))]   # a^(2k+1)
        for n in names:
            p.var(n, 1, os.environ.get("PGEN_INV_HOME", "A"))
        vr = "inv_r_" + tag
        p.var(vr)
        a2 = p.sqr(a)
        t = a
        for k, n in enumerate(names):
            if k:
                t = p.mul(t, a2)
            p.set(n, t)
        p.set(vr, p.get(names[(wins[0][1] - 1) // 2]))
        for nsq, val in wins[1:]:
            with p.loop(nsq):
                p.set(vr, p.sqr(p.get(vr)))
            p.set(vr, p.mul(p.get(vr), p.get(names[(val - 1) // 2])))
        if tail:
            with p.loop(tail):
                p.set(vr, p.sqr(p.get(vr)))
        return p.get(vr)

    def inv2(self, a, tag):  # fq2.rs:138-155
        p = self.p
        if self.fe_split == "inv":
            t = p.load(12)
        else:
            n = p.sop(a[0], a[0], a[1], a[1])
            if self.fe_split == "norm":
                raise NormStop(n)
            t = self.inv_fq(n, tag)
        return (p.mul(a[0], t), p.mul(p.neg(a[1]), t))

    def inv6(self, a, tag):  # fq6.rs:250-301
        t = self
        c0 = t.red2(t.sub2(t.sqr2(a[0]), t.mul2(t.xi(a[2]), a[1])))
        c1 = t.red2(t.sub2(t.red2(t.xi(t.sqr2(a[2]))), t.mul2(a[0], a[1])))
        c2 = t.red2(t.sub2(t.sqr2(a[1]), t.mul2(a[0], a[2])))
        s = t.red2(t.add2(t.xi(t.add2(t.mul2(a[2], c1), t.mul2(a[1], c2))), t.mul2(a[0], c0)))
        i = t.inv2(s, tag)
        return (t.mul2(i, c0), t.mul2(i, c1), t.mul2(i, c2))

    def inv12(self, a, tag="f"):  # fq12.rs:132-148
        t = self
        s = t.red6(t.sub6(t.mul6(a[0], a[0]), t.mul_v(t.mul6(a[1], a[1]))))
        i = t.inv6(s, tag)
        return (t.mul6(a[0], i), t.red6(t.neg6(t.mul6(a[1], i))))


# ======================= variables of tower values =======================
def names12(prefix):
    return ["%s%d" % (prefix, i) for i in range(12)]


def flat12(f):
    return [x for c6 in f for c2 in c6 for x in c2]


def unflat12(xs):
    xs = list(xs)
    return (((xs[0], xs[1]), (xs[2], xs[3]), (xs[4], xs[5])),
            ((xs[6], xs[7]), (xs[8], xs[9]), (xs[10], xs[11])))


def declare12(p, prefix, home=None):
    """home: preferred storage tier of the 12 variables ("A", "L" or "M")"""
    for n in names12(prefix):
        p.var(n, 1, home)


def set12(p, prefix, f):
    for n, v in zip(names12(prefix), flat12(f)):
        p.set(n, v)


def get12(p, prefix):
    return unflat12(p.get(n) for n in names12(prefix))


# ======================= lazy reduction (wide values) =======================
class Wide:
    """A double-width unreduced value lo + hi 2^392 (two DSL halves) with a
    bound vb on its value and `top` on hi's limb 13 (the subtraction
    constants need it)."""
    __slots__ = ("lo", "hi", "vb", "top")

    def __init__(self, lo, hi, vb, top):
        self.lo, self.hi, self.vb, self.top = lo, hi, vb, top


_WSUB = {}


def wide_sub_constant(ulo, uhi, top):
    """C = C_lo + C_hi 2^392 = k q with C_lo limbs >= ulo (2^28-1), C_hi limbs
    >= uhi (2^28-1) below limb 13 and >= top there: subtracting a wide value of
    those limb bounds half by half never goes negative, and C = 0 mod q."""
    key = (ulo, uhi, top)
    if key not in _WSUB:
        M = (1 << 28) - 1
        lo = [ulo * M] * 14
        hi = [uhi * M] * 13 + [top]
        val = lambda ls: sum(c << (28 * i) for i, c in enumerate(ls))
        minv = val(lo) + (val(hi) << 392)
        k = -(-minv // Q)
        d = k * Q - minv
        clo = [lo[i] + ((d >> (28 * i)) & M) for i in range(13)] + [lo[13] + (d >> (28 * 13))]
        assert val(clo) + (val(hi) << 392) == k * Q
        assert all(x < (1 << 32) for x in clo + hi)
        _WSUB[key] = (clo, hi, k * Q)
    return _WSUB[key]


class TowerLazy(Tower):
    """Tower with lazy reduction: Fq2 products are formed as wide (unreduced)
    values and combined before ONE Montgomery reduction per output Fq --
    Karatsuba at the Fq2 and Fq6 levels without paying a reduction per
    partial product.  Same field values as Tower (every output is a field
    element of the same class; canonical at the ABI), fewer multiply-
    accumulates: a wide product is 196 MACs, a reduction 196 + 27."""

    # ---- wide Fq ----
    def w_sop(self, *args):
        lo, hi = self.p.wsop(*args)
        vb = sum((a.vb * 2 * Q) * (b.vb * 2 * Q) for a, b in zip(args[0::2], args[1::2]))
        return Wide(lo, hi, vb, (vb - 1) >> 756)

    def w_norm(self, a):
        if a.lo.u == 1 and a.hi.u == 1:
            return a
        lo, hi = self.p.wnorm(a.lo, a.hi)
        return Wide(lo, hi, a.vb, (a.vb - 1) >> 756)

    @staticmethod
    def _wu(a):
        return max(a.lo.u, a.hi.u)

    def w_add(self, a, b):
        p = self.p
        if self._wu(a) + self._wu(b) > 12:
            a, b = (self.w_norm(a), b) if self._wu(a) >= self._wu(b) else (a, self.w_norm(b))
        if self._wu(a) + self._wu(b) > 12:
            a, b = self.w_norm(a), self.w_norm(b)
        return Wide(p.add(a.lo, b.lo), p.add(a.hi, b.hi), a.vb + b.vb, a.top + b.top)

    def w_sub(self, a, b):
        p = self.p
        if self._wu(b) > 3:
            b = self.w_norm(b)
        if self._wu(a) + self._wu(b) + 1 > 12:
            a = self.w_norm(a)
        clo, chi, cv = wide_sub_constant(b.lo.u, b.hi.u, b.top)
        return Wide(p.csub(a.lo, b.lo, clo), p.csub(a.hi, b.hi, chi), a.vb + cv, a.top + chi[13])

    def w_red(self, a):
        bound = a.vb // (1 << 392) + 1 + Q        # (W + m q) / 2^392 < W / 2^392 + q
        u = -(-bound // (2 * Q))
        r = self.p.wred(a.lo, a.hi, u)
        return r if u <= 2 else self.p.red(r)

    # ---- wide Fq2 ----
    def w_mul2(self, a, b):
        """Fq2 product, wide: Karatsuba (3 products) when the operand sums fit
        the column bound, else schoolbook (4 products in two 2-term sums)"""
        p = self.p
        ua0, ua1, ub0, ub1 = a[0].u, a[1].u, b[0].u, b[1].u
        if (ua0 + ua1) * (ub0 + ub1) <= 17:
            p0 = self.w_sop(a[0], b[0])
            p1 = self.w_sop(a[1], b[1])
            p2 = self.w_sop(p.add(a[0], a[1]), p.add(b[0], b[1]))
            return (self.w_sub(p0, p1), self.w_sub(p2, self.w_add(p0, p1)))
        if self.nu(a[1]) * ub1 <= ua1 * self.nu(b[1]):
            c0 = self.w_sop(a[0], b[0], p.neg(a[1]), b[1])
        else:
            c0 = self.w_sop(a[0], b[0], a[1], p.neg(b[1]))
        return (c0, self.w_sop(a[0], b[1], a[1], b[0]))

    def w_sqr2(self, a):
        p = self.p
        if (a[0].u + a[1].u) * (a[0].u + self.nu(a[1])) <= 17:
            c0 = self.w_sop(p.add(a[0], a[1]), p.sub(a[0], a[1]))
        else:
            c0 = self.w_sop(a[0], a[0], p.neg(a[1]), a[1])
        return (c0, self.w_sop(p.dbl(a[0]), a[1]))

    def w_add2(self, a, b): return (self.w_add(a[0], b[0]), self.w_add(a[1], b[1]))
    def w_sub2(self, a, b): return (self.w_sub(a[0], b[0]), self.w_sub(a[1], b[1]))
    def w_xi(self, a): return (self.w_sub(a[0], a[1]), self.w_add(a[0], a[1]))
    def w_red2(self, a): return (self.w_red(a[0]), self.w_red(a[1]))

    # ---- overrides ----
    def mul2(self, a, b):  # fq2.rs:123-136
        ua, ub = self.u2(a), self.u2(b)
        if (a[0].u + a[1].u) * (b[0].u + b[1].u) <= 17:
            return self.w_red2(self.w_mul2(a, b))
        return Tower.mul2(self, a, b)

    def mul6(self, a, b):  # fq6.rs:199-248, Karatsuba, one reduction per output Fq
        t = self
        assert self.u6(a) <= 2 and self.u6(b) <= 2
        s12 = (t.lim1(t.add2(a[1], a[2])), t.lim1(t.add2(b[1], b[2])))
        v1 = t.w_mul2(a[1], b[1])
        v2 = t.w_mul2(a[2], b[2])
        t0 = t.w_mul2(*s12)
        c0 = t.w_sub2(t0, t.w_add2(v1, v2))
        v0 = t.w_mul2(a[0], b[0])
        c0 = t.w_red2(t.w_add2(t.w_xi(c0), v0))
        t2 = t.w_mul2(t.lim1(t.add2(a[0], a[2])), t.lim1(t.add2(b[0], b[2])))
        c2 = t.w_red2(t.w_add2(t.w_sub2(t2, t.w_add2(v0, v2)), v1))
        t1 = t.w_mul2(t.lim1(t.add2(a[0], a[1])), t.lim1(t.add2(b[0], b[1])))
        c1 = t.w_red2(t.w_add2(t.w_sub2(t1, t.w_add2(v0, v1)), t.w_xi(v2)))
        return (t.lim1(c0), t.lim1(c1), t.lim1(c2))

    def lim1(self, a):
        """Karatsuba operands: the Fq2-level sums of these feed products"""
        return a if self.u2(a) <= 2 else self.red2(a)

    def mul_by_01(self, a, c0, c1):  # fq6.rs:68-109
        t = self
        a_a = t.w_mul2(a[0], c0)
        b_b = t.w_mul2(a[1], c1)
        t1 = t.w_mul2(c1, t.lim1(t.add2(a[1], a[2])))
        r0 = t.w_red2(t.w_add2(t.w_xi(t.w_sub2(t1, b_b)), a_a))
        t3 = t.w_mul2(c0, t.lim1(t.add2(a[0], a[2])))
        r2 = t.w_red2(t.w_add2(t.w_sub2(t3, a_a), b_b))
        t2 = t.w_mul2(t.lim1(t.add2(c0, c1)), t.lim1(t.add2(a[0], a[1])))
        r1 = t.w_red2(t.w_sub2(t2, t.w_add2(a_a, b_b)))
        return (t.lim1(r0), t.lim1(r1), t.lim1(r2))

    def fq4_sqr(self, a, b):
        t = self
        t0 = t.w_sqr2(a)
        t1 = t.w_sqr2(b)
        r0 = t.w_red2(t.w_add2(t.w_xi(t1), t0))
        t2 = t.w_sqr2(t.lim1(t.add2(a, b)))
        r1 = t.w_red2(t.w_sub2(t2, t.w_add2(t0, t1)))
        return t.lim1(r0), t.lim1(r1)

    def ksqr(self, g):
        """Tower.ksqr with each half's x^2 + xi y^2 and 2 x y formed from wide
        squares, one reduction per output Fq (PGEN_KSQR_LAZY=0: Tower.ksqr)"""
        if os.environ.get("PGEN_KSQR_LAZY", "1") != "1":
            return Tower.ksqr(self, g)
        t = self
        a1, a2, b0, b2 = g

        def half(x, y, z, zy, xi_on_cross):
            sx, sy = t.w_sqr2(x), t.w_sqr2(y)
            s = t.lim1(t.w_red2(t.w_add2(sx, t.w_xi(sy))))
            sxy = t.w_sqr2(t.lim1(t.add2(x, y)))
            c = t.lim1(t.w_red2(t.w_sub2(sxy, t.w_add2(sx, sy))))
            if xi_on_cross:
                c = t.red2(t.xi(c))
            nz = t.red2(t.add2(t.dbl2(t.sub2(s, z)), s))
            nzy = t.red2(t.add2(t.dbl2(t.add2(c, zy)), c))
            return nz, nzy

        na2, nb0 = half(a1, b2, a2, b0, True)
        na1, nb2 = half(b0, a2, a1, b2, False)
        return (na1, na2, nb0, nb2)


class TowerLazySq(TowerLazy):
    """Only the Fq4 squaring of the cyclotomic square is lazy: its three Fq2
    squares stay wide and each output Fq is reduced once -- the one override
    that lowers the final exponentiation's instruction count
    (tools/pgen/lazy_explore.py); every other product as in Tower."""
    mul2 = Tower.mul2
    mul6 = Tower.mul6
    mul_by_01 = Tower.mul_by_01
