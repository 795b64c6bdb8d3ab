"""The tower on a lane pair: lane r holds coordinate r of every Fq2 value
(a "distributed" Fq2 is one DSL Val); Fq values outside Fq2 (P's
coordinates, the norm inverted in Fq2 inversion) are replicated on both
lanes.  Fq6 / Fq12 code is inherited unchanged from tower.Tower -- only the
Fq2 primitives are redefined here, each as per-lane operations plus the
partner exchange (swap: DPP quad_perm [1,0,3,2]) and lane selects.

Products: lane 0 computes c0 = a0 b0 - a1 b1, lane 1 c1 = a0 b1 + a1 b0,
both as the same two-term leaf sop(X, b, Z, b'), with b' = swap(b) and
X = (a0 | a0), Z = (-a1 | a1) formed by selects.  Every field value equals
the one-lane tower's (checked by dsl.evaluate against the C oracle).
"""
import os

from dsl import SUBCU

PREP_REUSE = os.environ.get("PGEN_PREP_REUSE", "1") == "1"
DPP_ADD = os.environ.get("PGEN_DPP_ADD", "1") == "1"
SQR_NORM = os.environ.get("PGEN_SQR_NORM", "1") == "1"
PAIR_SUM = os.environ.get("PGEN_PAIR_SUM", "0") == "1"   # measured: more live pairs, more spills
# mul2's operand pair by a DPP broadcast and a fused negate + DPP select (42
# instructions) instead of swap, negate and two selects (56)
PAIR_DPP = os.environ.get("PGEN_PAIR_DPP", "1") == "1"
# sqr2 with a signed second operand (a0 - a1 | a0): three exchange ops instead
# of four (dsl.Prog.pdiff / _ssop).  Measured off: the product adds q to stay
# positive, so its value bound is 2 and the sums after it need full reductions
# where carry passes did (FE2 +0.1 % instructions, ML2p -0.14 %); built for
# A/B as build_gen "ml2ps"
SQR_SIGNED = os.environ.get("PGEN_SQR_SIGNED", "0") == "1"
MUL2_USES = {}       # value id -> mul2 operand uses, from a first build (two_pass)
MUL2_COUNT = None
SWAPPED = set()      # value ids whose partner swap a first build formed (outside xi)
XI_DPP = True        # xi by dppadd (two_pass(xi_dpp=...): measured per kernel)


def two_pass(progf, xi_dpp=True):
    """build a lane-pair program twice: the first build counts how often each
    value is a mul2 operand (value ids are deterministic), the second lets
    mul2 form the (x, z) pair of the more used operand"""
    global MUL2_USES, MUL2_COUNT

    def f():
        global MUL2_USES, MUL2_COUNT, SWAPPED, XI_DPP
        import dsl
        XI_DPP = xi_dpp
        MUL2_USES, MUL2_COUNT, SWAPPED = {}, {}, set()
        seen = set()
        swap0 = dsl.Prog.swap

        def swap(self, a):
            seen.add(a.id)
            return swap0(self, a)
        dsl.Prog.swap = swap
        try:
            progf()
        finally:
            dsl.Prog.swap = swap0
        MUL2_USES, MUL2_COUNT, SWAPPED = MUL2_COUNT, None, seen
        try:
            return progf()
        finally:
            MUL2_USES, SWAPPED, XI_DPP = {}, set(), True
    return f
from tower import Tower


class Tower2(Tower):
    def __init__(self, p):
        super().__init__(p)
        self.sums = {}    # value id -> (a, b): the value is a + b (add2, or lim2 / red2 of such a sum)
        self.pairs = {}   # (block, value id) -> mul2's operand pair (x, z) formed in that block

    # ---------------- distributed Fq2 ----------------
    def add2(self, a, b):
        r = self.p.add(a, b)
        if PAIR_SUM:
            self.sums[r.id] = (a, b)
        return r
    def sub2(self, a, b): return self.p.sub(a, b)
    def neg2(self, a): return self.p.neg(a)
    def dbl2(self, a): return self.p.add(a, a)
    def red2(self, a):
        r = self.p.red(a)
        if r is not a and a.id in self.sums:
            self.sums[r.id] = self.sums[a.id]
        return r
    def u2(self, a): return a.u

    def xi(self, a):
        """(a0 - a1, a0 + a1): mine + the partner's entry of conj(a) = (a0 | -a1),
        one v_add_u32_dpp per limb"""
        p = self.p
        # one v_add_u32_dpp per limb unless a's swap is formed anyway (by mul2 or
        # sqr2 of a, counted by the first build of two_pass): then 3 ops over it
        if DPP_ADD and XI_DPP and a.id not in SWAPPED:
            return p.dppadd(self.conj2(a), a, (1, 0))
        o = p.swap(a)
        return p.add(a, p.sel(p.neg(o), o))

    def conj2(self, a):
        p = self.p
        return p.sel(a, p.neg(a))

    def _sqr_fits(self, vb):
        p = self.p
        cv = p.sub_bounds((1, vb) if vb > 1 else 1)[1]
        return 2 * vb * max(vb + cv, vb) <= 600

    def _prepped(self, a):
        """a's operand pair (x, z) of mul2 is already formed in this block"""
        memo = self.p.cur.__dict__.get("memo", {})
        return (not PAIR_DPP and ("swap", (a.id,), None) in memo) or (id(self.p.cur), a.id) in self.pairs

    def _pair_direct(self, a):
        p = self.p
        if PAIR_DPP:
            # a0 on both lanes (one DPP broadcast); -a1 | a1 (a sub and a DPP select)
            return p.bcast(a, 0), p.pairz(a)
        oa = p.swap(a)
        return p.sel(a, oa), p.sel(p.neg(oa), a)     # a0 on both lanes; -a1 | a1

    def _summed(self, a):
        """the pairs of a's summands, both formed already in this block, or None"""
        s = self.sums.get(a.id) if PAIR_SUM else None
        if s is None or not all((id(self.p.cur), v.id) in self.pairs for v in s):
            return None
        return [self.pairs[(id(self.p.cur), v.id)] for v in s]

    def _pair_cost(self, a):
        if self._prepped(a):
            return 0
        return 28 if self._summed(a) is not None else (42 if PAIR_DPP else 56)

    def _pair_fits(self, x, z, b):
        p = self.p
        if x.u * b.u + z.u * b.u > 17:
            return False
        return not p.use_norm or x.vb * b.vb + z.vb * b.vb <= 600

    def pair(self, a, b):
        """mul2's operand pair of a (against partner operand b): the pair of a
        sum is the sum of its summands' pairs (x and z are linear in a) when
        those are formed and the product's bounds hold -- 2 adds instead of a
        swap, a negation and two selects"""
        p = self.p
        key = (id(p.cur), a.id)
        if key in self.pairs:
            return self.pairs[key]
        s = self._summed(a)
        r = None
        if s is not None:
            (x0, z0), (x1, z1) = s
            x, z = p.add(x0, x1), p.add(z0, z1)
            if self._pair_fits(x, z, b):
                r = (x, z)
        if r is None:
            r = self._pair_direct(a)
        self.pairs[key] = r
        return r

    def _fits(self, a, b):
        p = self.p
        zu = max(p.neg_u(a), a.u)
        if a.u * b.u + zu * b.u > 17:
            return False
        if p.use_norm:
            zv = max(p.sub_bounds(p.sub_key(a))[1], a.vb)
            return a.vb * b.vb + zv * b.vb <= 600
        return True

    def mul2(self, a, b):
        p = self.p
        if SUBCU[a.u] * b.u > a.u * SUBCU[b.u]:
            a, b = b, a
        # the (x, z) pair costs 42 (56) instructions, the partner swap of b 14: let
        # the operand whose pair is already formed be a -- or, neither being
        # formed, the one more products will use (MUL2_USES, a first build's
        # count) -- if the bounds allow
        if PREP_REUSE and self._fits(b, a):
            ca, cb = self._pair_cost(a), self._pair_cost(b)
            if cb < ca or (cb == ca and cb and MUL2_USES.get(b.id, 0) > MUL2_USES.get(a.id, 0)):
                a, b = b, a
        if MUL2_COUNT is not None:
            MUL2_COUNT[a.id] = MUL2_COUNT.get(a.id, 0) + 1
            MUL2_COUNT[b.id] = MUL2_COUNT.get(b.id, 0) + 1
        x, z = self.pair(a, b)
        ob = p.swap(b)
        return p.sop(x, b, z, ob)     # lane 0: a0 b0 - a1 b1; lane 1: a0 b1 + a1 b0

    def sqr2(self, a):
        """lane 0: (a0 + a1)(a0 - a1); lane 1: 2 a0 a1"""
        p = self.p
        if a.u > 1:
            # a carry pass (value unchanged) where the product's value bound still
            # holds for it: x = o + a0 has 2 vb, y = a - o about 2.2 vb + 1
            if SQR_NORM and p.use_norm and a.u <= 15 and self._sqr_fits(a.vb):
                a = p.norm_only(a)
            else:
                a = p.red(a)
        if SQR_SIGNED:
            # lane 0: (a1 + a0)(a0 - a1), lane 1: (2 a1) a0; the product adds q
            # (signed operand), so its value bound is 2
            x = p.dppadd(a, a, (1, 1))    # a1 + a0 | 2 a1
            return p.mul(x, p.pdiff(a))
        o = p.swap(a)
        if DPP_ADD:
            x = p.dppadd(a, o, (0, 0))    # o + a0: a0 + a1 | 2 a0, one v_add_u32_dpp per limb
        else:
            x = p.add(o, p.sel(a, o))     # a0 + a1 | 2 a0
        y = p.sel(p.sub(a, o), a)     # a0 - a1 | a1
        return p.mul(x, y)

    def mul_fq(self, a, b):
        return self.p.mul(a, b)       # b replicated

    def lim2(self, a):
        return a if a.u <= 2 else self.red2(a)

    def const2(self, c):
        p = self.p
        return p.sel(p.const(c[0]), p.const(c[1]))

    def one2(self):
        return self.const2((1, 0))

    # ---------------- Karabina decompression (tower.Tower, lane pairs) ----------------
    def kdec_numden(self, g):
        """Tower.kdec_numden on distributed Fq2: the b0 == 0 test reads both
        coordinates (this lane's and the partner's), so both lanes of a pair
        take the same branch; w = 3 a1 a2 - b0 b2 as two Fq2 products"""
        t, p = self, self.p
        a1, a2, b0, b2 = g
        s1 = t.sqr2(a1)
        num1 = t.red2(t.sub2(t.add2(t.add2(t.dbl2(s1), s1), t.xi(t.sqr2(b2))), t.dbl2(a2)))
        den1 = t.red2(t.dbl2(t.dbl2(b0)))
        num2 = t.red2(t.dbl2(t.mul2(a1, b2)))
        den2 = t.red2(a2)
        zb = p.red_full(b0)
        z = [zb, p.swap(zb)]
        num = p.selz(z, num2, num1)
        den = p.selz(z, den2, den1)
        a13 = t.lim2(t.add2(t.dbl2(a1), a1))
        w = t.red2(t.sub2(t.mul2(a13, a2), t.mul2(b0, b2)))
        return num, den, w

    def inv2_direct(self, a, tag):
        return self.inv2(a, tag)

    # ---------------- inversion ----------------
    def inv2(self, a, tag):
        """fq2.rs:138-155: the norm a0^2 + a1^2 is formed on both lanes and
        inverted redundantly (replicated Fq)"""
        p = self.p
        sq = p.mul(a, a)
        t = self.inv_fq(p.red(p.add(sq, p.swap(sq))), tag)
        return p.mul(self.conj2(a), t)
