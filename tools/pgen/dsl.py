"""Tracing DSL for the pairing kernels over the lazy 28-bit-limb field.

A kernel is built by running Python code that calls Prog methods; every
call appends an Op to the current Block and returns an SSA value `Val`
carrying its static bound u (every limb <= u (2^28-1), value < u 2q; see
pairing_amd/csrc/fl.h).  Long-lived state crosses loop / branch
boundaries through named variables (getvar / setvar), which the register
allocator pins to fixed homes.

`evaluate()` interprets a Prog on concrete inputs with the exact limb
semantics of the emitted instructions (column-accumulator Montgomery
products, the one-pass red(), limb-wise add/sub), asserting every bound as
it goes -- the golden model the instruction-level simulator and the GPU are
compared against, and itself compared against the C oracle.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from gen_consts import Q  # noqa: E402
import gen_fl  # noqa: E402

NL, LB, MASK = gen_fl.NL, gen_fl.LB, gen_fl.MASK
R = 1 << (NL * LB)
QL = gen_fl.limbs(Q)
QINV28 = gen_fl.QINV
KQ = gen_fl.KQ
SUBC = {}
SUBCU = {}
for _ub in range(1, gen_fl.U_MAX_SUB + 1):
    SUBC[_ub], SUBCU[_ub] = gen_fl.sub_constant(_ub)
U_MAX = 16
COL_BOUND = 17
# Value bounds (Val.vb, in units of 2q) are tracked apart from limb bounds (Val.u):
# a Montgomery product of sum a_i b_i is < 2q whenever sum vb_a vb_b 4q^2 < q 2^392,
# i.e. sum vb_a vb_b < 2^392 / 4q ~ 630 (VB_PROD below keeps a margin), whatever
# the limb bounds (those only guard the 64-bit columns).  So a sum that only has
# to feed products needs its LIMBS brought back below 2^28 ("norm": a carry pass,
# 39 instructions), not its value below 2q ("red": quotient estimate + signed
# k q subtraction, 62 instructions).
VB_PROD = 600
VB_RED = 64        # red's quotient estimate needs the value below 2^388
VN = int(os.environ.get("PGEN_VN", "6"))   # norm instead of red while vb <= VN


def _val_of(limbs):
    return sum(int(x) << (LB * i) for i, x in enumerate(limbs))


class _SubTables(dict):
    """SUBC[ub] (int: the classic tables, subtrahend bounds u = vb = ub) and
    SUBC[(u, vb)] (norm programs: a subtrahend of limb bound u whose value bound
    vb exceeds u), built on demand; SUBCL / SUBCV: limb / value bound of C"""
    def __missing__(self, key):
        c, ul, uv = gen_fl.sub_constant2(*key)
        self[key] = c
        SUBCL[key], SUBCV[key] = ul, uv
        return c


SUBCL, SUBCV = {}, {}
SUBC = _SubTables(SUBC)
for _ub in list(SUBC):
    _c, SUBCL[_ub], SUBCV[_ub] = gen_fl.sub_constant2(_ub, _ub)
    assert _c == SUBC[_ub]


def to_mont_limbs(x):
    """field value -> canonical Fl limbs (x R mod q)"""
    return tuple(gen_fl.limbs(x * R % Q))


def val_of(limbs):
    return sum(int(x) << (LB * i) for i, x in enumerate(limbs))


class Val:
    """An SSA value of 14 limbs.  `half`: one half (limbs 0..13 or 14..27) of a
    double-width unreduced product ("wide" value, see Prog.wsop): only its
    limb bound u is tracked here, the value bound of the pair is tracked by
    the code that builds it (tower.py Wide)."""
    __slots__ = ("id", "u", "half", "vb", "sgn")

    def __init__(self, id_, u, half=False, vb=None):
        self.id, self.u, self.half = id_, u, half
        self.vb = u if vb is None else vb     # value < vb 2q (full values)
        # signed (Prog.pdiff): limbs in (-u MASK, u MASK], |value| < vb 2q; only
        # the second operand of a product may be signed (Prog.mul -> "ssop")
        self.sgn = False

    def __repr__(self):
        return "v%d/u%d%s%s" % (self.id, self.u, "" if self.vb == self.u else "/vb%d" % self.vb,
                                "h" if self.half else "")


class Op:
    __slots__ = ("kind", "dst", "srcs", "imm", "dst2")

    def __init__(self, kind, dst, srcs, imm=None, dst2=None):
        self.kind, self.dst, self.srcs, self.imm, self.dst2 = kind, dst, srcs, imm, dst2

    def __repr__(self):
        return "%s %s%s <- %s %s" % (self.kind, self.dst, "" if self.dst2 is None else ",%r" % self.dst2, self.srcs,
                                     "" if self.imm is None else self.imm)


class Block:
    def __init__(self):
        self.items = []


class Loop:
    """body runs `trips` times; counter i = trips-1 .. 0 (bit index for If)"""

    def __init__(self, trips):
        self.trips = trips
        self.body = Block()


class If:
    """body runs when (mask >> loop.i) & 1"""

    def __init__(self, mask, loop):
        self.mask, self.loop = mask, loop
        self.body = Block()


class Var:
    def __init__(self, name, u, home, vb=None):
        self.name, self.u, self.home = name, u, home
        self.vb = u if vb is None else vb


class Prog:
    def __init__(self, name, lanes=1, use_norm=False):
        self.name = name
        self.lanes = lanes      # 2: a lane pair shares each pairing (tower2.py)
        self.use_norm = use_norm  # red() may carry-normalize (see VB_PROD)
        self.root = Block()
        self.cur = self.root
        self.nval = 0
        self.vars = {}
        self.inputs = []   # (name, kind): kernel inputs, see kernels.py
        self.stack = []

    # ---- plumbing ----
    def _val(self, u, half=False, vb=None):
        assert 1 <= u <= U_MAX, "bound %d out of range" % u
        v = Val(self.nval, u, half, vb)
        assert half or 1 <= v.vb <= VB_RED * 16, "value bound %d out of range" % v.vb
        self.nval += 1
        return v

    def _op(self, kind, srcs, u, imm=None, vb=None):
        half = any(x.half for x in srcs) and kind in ("add", "csub", "getvar")
        v = self._val(u, half, vb) if u else None
        self.cur.items.append(Op(kind, v, list(srcs), imm))
        return v

    @staticmethod
    def _full(*vals):
        assert not any(v.half for v in vals), "field op on a wide half"
        assert not any(v.sgn for v in vals), "a signed value is only a product's second operand"

    # ---- field ops ----
    def mul(self, a, b):
        if b.sgn:
            return self._ssop(a, b)
        self._full(a, b)
        assert a.u * b.u <= COL_BOUND, "mul bound %d*%d" % (a.u, b.u)
        assert a.vb * b.vb <= VB_PROD, "mul value bound %d*%d" % (a.vb, b.vb)
        return self._op("sop", [a, b], 1)

    def _ssop(self, a, b):
        """a b with b signed (pdiff): the leaf's products by v_mad_i64_i32 into a
        signed accumulator, arithmetic carries, and q added by the last
        Montgomery digit (m_13 + 2^28: + R q before the division), so the
        result (s + m q) / R + q is positive: value in (q - e, 2q + e) for the
        bounds below -- u = 1, vb = 2 (emit.Emitter.emit_sop signed=True;
        exact limbs: mont_sop_signed)"""
        self._full(a)
        assert not b.half
        assert a.u * b.u <= 8, "signed product bound %d*%d (the accumulator has 63 bits)" % (a.u, b.u)
        assert a.u <= 8, "a's limbs must read as signed 32-bit"
        # |a b| / R < 4 a.vb b.vb q^2 / R ~ 0.0016 a.vb b.vb q: the result stays in
        # (0, 4q) while a.vb b.vb < 629
        assert a.vb * b.vb <= VB_PROD, "signed product value bound %d*%d" % (a.vb, b.vb)
        return self._op("ssop", [a, b], 1, vb=2)

    def sop(self, a, b, c, d):
        self._full(a, b, c, d)
        assert a.u * b.u + c.u * d.u <= COL_BOUND, "sop bound %d*%d+%d*%d" % (a.u, b.u, c.u, d.u)
        assert a.vb * b.vb + c.vb * d.vb <= VB_PROD, "sop value bound"
        return self._op("sop", [a, b, c, d], 1)

    def sopn(self, args):
        """sum a_i b_i over the pairs (a0, b0, a1, b1, ...): one product leaf"""
        self._full(*args)
        assert len(args) % 2 == 0 and args
        assert sum(a.u * b.u for a, b in zip(args[0::2], args[1::2])) <= COL_BOUND, "sopn bound"
        assert sum(a.vb * b.vb for a, b in zip(args[0::2], args[1::2])) <= VB_PROD, "sopn value bound"
        return self._op("sop", list(args), 1)

    def sqr(self, a):
        self._full(a)
        assert a.u <= 3, "sqr bound %d" % a.u
        assert a.vb * a.vb <= VB_PROD, "sqr value bound %d" % a.vb
        return self._op("sqr", [a], 1)

    def inv(self, a):
        """a^-1 in the Fl domain (0 -> 0) as ONE op.  The cooperative kernels
        (coop.py, kernels_coop.hip) run it on the 12-word core's binary GCD
        (bgcd.h); the one-lane generated kernels use binv() (or Tower.inv_fq's
        Fermat chain with PGEN_BINV=0)."""
        self._full(a)
        return self._op("inv", [a], 1)

    def binv(self, a):
        """a^-1 in the Fl domain (0 -> 0) by the in-kernel binary GCD of the
        one-lane generated kernels (emit.Emitter.emit_binv; exact output limbs:
        binv_limbs below).  u = 1, value < 2q, not canonical."""
        self._full(a)
        assert a.vb <= VB_RED, "binv value bound %d" % a.vb
        return self._op("binv", [a], 1)

    def selz(self, tests, a, b):
        """a where every test value is 0 mod q, else b (lane-wise select).  The
        tests must be fully reduced (u = vb = 1: limbs < 2^28, value < 2q, so
        zero mod q means the limbs are those of 0 or of q)."""
        self._full(a, b, *tests)
        assert all(t.u == 1 and t.vb == 1 for t in tests), "selz tests must be reduced"
        return self._op("selz", list(tests) + [a, b], max(a.u, b.u), imm=len(tests), vb=max(a.vb, b.vb))

    def red_full(self, a):
        """the full reduction (value < 2q, limbs < 2^28) whatever the value bound"""
        self._full(a)
        if a.u == 1 and a.vb == 1:
            return a
        assert a.vb <= VB_RED, "red value bound %d" % a.vb
        return self._cse("red", [a], 1, vb=1)

    # ---- wide (double-width, unreduced) values: lazy reduction ----
    def wsop(self, *args):
        """sum a_i b_i over the pairs (a0, b0, a1, b1, ...) as a 28-limb
        normalized integer, NOT reduced: returns its halves (lo, hi).  Costs
        the products of a sop without its Montgomery reduction."""
        self._full(*args)
        assert len(args) % 2 == 0 and args
        assert sum(a.u * b.u for a, b in zip(args[0::2], args[1::2])) <= COL_BOUND, "wsop bound"
        assert sum(a.vb * b.vb for a, b in zip(args[0::2], args[1::2])) <= VB_PROD, "wsop value bound"
        lo, hi = self._val(1, True), self._val(1, True)
        self.cur.items.append(Op("wsop", lo, list(args), dst2=hi))
        return lo, hi

    def wnorm(self, lo, hi):
        """carry-propagate a wide value: every limb < 2^28 again (u = 1)"""
        assert lo.half and hi.half
        nlo, nhi = self._val(1, True), self._val(1, True)
        self.cur.items.append(Op("wnorm", nlo, [lo, hi], dst2=nhi))
        return nlo, nhi

    def csub(self, a, b, climbs):
        """a + C - b limb-wise with an explicit constant C (limbs >= b's)"""
        ul = max(-(-c // MASK) for c in climbs)
        return self._op("csub", [a, b], a.u + ul, imm=tuple(climbs))

    def wred(self, lo, hi, u):
        """Montgomery reduction (lo + hi 2^392) / 2^392 mod q of a wide value;
        the caller proves the output bound u (checked by evaluate)."""
        assert lo.half and hi.half
        return self._op("wred", [lo, hi], u)

    def add(self, a, b):
        return self._op("add", [a, b], a.u + b.u, vb=None if a.half else a.vb + b.vb)

    def dbl(self, a):
        return self.add(a, a)

    def sub_key(self, b):
        """SUBC table for subtrahend b: limbs 0..12 need C_i >= b.u MASK, the top
        limb (< value / 2^364 < vb 2^18) needs C_13 >= vb 2^18"""
        if not self.use_norm or b.vb <= b.u:
            assert b.u in SUBCU, "subtrahend bound %d" % b.u
            return b.u
        return (b.u, b.vb)

    def sub_bounds(self, key):
        """(limb bound, value bound) of the constant C of table `key`"""
        SUBC[key]
        if not self.use_norm:
            return SUBCU[key], SUBCU[key]
        return SUBCL[key], SUBCV[key]

    def neg_u(self, b):
        return self.sub_bounds(self.sub_key(b))[0]

    def sub(self, a, b):
        self._full(a, b)
        key = self.sub_key(b)
        cu, cv = self.sub_bounds(key)
        return self._op("sub", [a, b], a.u + cu, imm=key, vb=None if not self.use_norm else a.vb + cv)

    def neg(self, b):
        self._full(b)
        key = self.sub_key(b)
        cu, cv = self.sub_bounds(key)
        return self._cse("neg", [b], cu, imm=key, vb=None if not self.use_norm else cv)

    def red(self, a):
        """bring a to limb bound 1: a carry pass ("norm", value unchanged) while
        the value bound stays small, else the full reduction (value < 2q)"""
        self._full(a)
        if a.u == 1 and a.vb <= (VN if self.use_norm else 1):
            return a
        if self.use_norm and a.u <= 15 and a.vb <= VN:
            return self._cse("norm", [a], 1, vb=a.vb)
        assert a.vb <= VB_RED, "red value bound %d" % a.vb
        return self._cse("red", [a], 1, vb=1)

    def norm_only(self, a):
        """the carry pass whatever VN says (limbs back below 2^28, value bound
        unchanged): for callers that check the bound their use needs"""
        self._full(a)
        assert self.use_norm and a.u <= 15
        if a.u == 1:
            return a
        return self._cse("norm", [a], 1, vb=a.vb)

    def _cse(self, kind, srcs, u, imm=None, vb=None):
        """pure ops on the same operands in the same block are computed once"""
        memo = self.cur.__dict__.setdefault("memo", {})
        key = (kind, tuple(v.id for v in srcs), imm)
        if key not in memo:
            memo[key] = self._op(kind, srcs, u, imm, vb)
        return memo[key]

    # ---- lane-pair ops (two-lane programs) ----
    def swap(self, a):
        """the partner lane's value (v_mov_b32_dpp quad_perm:[1,0,3,2])"""
        assert self.lanes == 2
        return self._cse("swap", [a], a.u, vb=a.vb)

    def dppadd(self, a, b, perm):
        """lane r: b + a of lane perm[r] of the pair (one v_add_u32_dpp per limb,
        quad_perm [perm0, perm1, perm0 + 2, perm1 + 2])"""
        assert self.lanes == 2
        self._full(a, b)
        return self._cse("dppadd", [a, b], a.u + b.u, imm=tuple(perm), vb=a.vb + b.vb)

    def sel(self, a, b):
        """lane 0 takes a, lane 1 takes b"""
        assert self.lanes == 2
        return self._cse("sel", [a, b], max(a.u, b.u), vb=max(a.vb, b.vb))

    def pdiff(self, a):
        """lane 0: a0 - a1 (its own a minus the partner's), lane 1: a0 (the
        partner's) -- SIGNED limbs, the second operand of an Fq2 squaring's
        product (tower2.Tower2.sqr2): a v_cndmask_b32_dpp (partner's a | 0) and
        a v_sub_u32_dpp (a0 - that) per limb"""
        assert self.lanes == 2
        self._full(a)
        v = self._cse("pdiff", [a], a.u, vb=a.vb)
        v.sgn = True
        return v

    def bcast(self, a, r):
        """lane r's value of a in both lanes of the pair (one v_mov_b32_dpp per
        limb, quad_perm [r, r, r + 2, r + 2])"""
        assert self.lanes == 2 and r in (0, 1)
        return self._cse("bcast", [a], a.u, imm=r, vb=a.vb)

    def pairz(self, a):
        """lane 0: -(lane 1's a) (C - a1, C the subtraction constant of a's
        bound), lane 1: its own a -- sel(neg(swap(a)), a) as one op: a v_sub_u32
        and a v_cndmask_b32_dpp (quad_perm swap, VCC = the odd-lane mask) per limb"""
        assert self.lanes == 2
        self._full(a)
        key = self.sub_key(a)
        cu, cv = self.sub_bounds(key)
        return self._cse("pairz", [a], max(cu, a.u), imm=key, vb=max(cv, a.vb) if self.use_norm else None)

    def const(self, x):
        """field element x (plain integer) as a canonical Fl constant"""
        return self._op("const", [], 1, imm=to_mont_limbs(x % Q))

    def const_limbs(self, limbs):
        return self._op("const", [], 1, imm=tuple(limbs))

    # ---- state ----
    def var(self, name, u=1, home=None):
        # under norm a variable may hold a carry-normalized value (bound VN;
        # PGEN_VARVB overrides it for A/B); set() fully reduces anything larger
        # (lane pairs: 5, so that x + y of two variables stays within the Fq2
        # squaring's product bound after a carry pass; tower2.Tower2.sqr2)
        vb = int(os.environ.get("PGEN_VARVB", str(VN if self.lanes == 1 else 5)))
        self.vars[name] = Var(name, u, home, max(u, vb) if self.use_norm else u)

    def get(self, name):
        var = self.vars[name]
        return self._op("getvar", [], var.u, imm=name, vb=var.vb)

    def set(self, name, v):
        assert v.u <= self.vars[name].u, "setvar %s: bound %d > %d" % (name, v.u, self.vars[name].u)
        if not v.half and v.vb > self.vars[name].vb:
            assert v.vb <= VB_RED
            v = self._cse("red", [v], 1, vb=1)
        assert v.half or v.vb <= self.vars[name].vb, "setvar %s: value bound %d" % (name, v.vb)
        self.cur.items.append(Op("setvar", None, [v], imm=name))

    # ---- cooperative macro operands (coop.py): value slots addressed by
    # (group, index); an arg is a stored field value of bound u, a ret stores
    # a value (bound 1) ----
    def arg(self, group, index, u=1):
        return self._op("arg", [], u, imm=(group, index))

    def ret(self, group, index, v):
        assert v.u == 1, "a macro output must be reduced (bound 1)"
        self.cur.items.append(Op("ret", None, [v], imm=(group, index)))

    # ---- kernel I/O (see kernels.py for the record layouts) ----
    def load(self, slot, slot1=None):
        """input Fq number `slot` of this lane's record (canonical, R = 2^384)
        -> Fl with R = 2^392 (u = 1): raw limbs times 2^400 mod q.  Two-lane
        programs: lane 1 reads `slot1` (default: the same slot)."""
        imm = slot if slot1 is None else (slot, slot1)
        raw = self._op("load_raw", [], 1, imm=imm)
        return self.mul(raw, self.const_limbs(gen_fl.limbs(pow(2, 400, Q))))

    def load_scaled(self, slot, c):
        """input Fq `slot` (raw ABI limbs, value x R) times the constant integer c
        in one product: x R c / R' (load() is c = 2^400, i.e. x R')"""
        raw = self._op("load_raw", [], 1, imm=slot)
        return self.mul(raw, self.const_limbs(gen_fl.limbs(c % Q)))

    # ---- a line table shared by every lane (one G2Prepared for the batch) ----
    def tload(self, j):
        """value j (0..5) of the current line of the kernel's line table: 14
        limbs read from a wave-uniform address (kcfg.MillerLoopSharedCfg), given
        as exact limbs (u = vb = 1, see kernels.miller_loop_shared_prog)"""
        return self._op("tload", [], 1, imm=j)

    def tnext(self):
        """advance the line table to the next line"""
        self.cur.items.append(Op("tnext", None, [], imm=None))

    def store(self, slot, v, slot1=None):
        """canonical output Fq `slot` (R = 2^384) of this lane (two-lane
        programs: lane 1 writes `slot1`)"""
        if slot1 is not None:
            slot = (slot, slot1)
        w = self.mul(self.red(v), self.const_limbs(gen_fl.limbs(pow(2, 384, Q))))
        self.cur.items.append(Op("store_raw", None, [w], imm=slot))

    # ---- control ----
    def loop(self, trips):
        return _Ctx(self, Loop(trips))

    def if_bit(self, mask, loop):
        return _Ctx(self, If(mask, loop))


def fuse_adds(prog):
    """Rewrite, per block, adds whose operands are single-use adds / doublings of
    the same block (values and bounds stay those of the outer op; the inner
    value disappears):
      add(x, x) of a single-use shl(y, s) or add(y, y)  -> shl(y, s + 1)   v_lshlrev_b32
      add(shl(x, s), y) / add(add(x, x), y)             -> shladd(x, y; s) v_lshl_add_u32
      add(add(a, b), c)                                 -> add3(a, b, c)   v_add3_u32
    Returns the number of rewrites."""
    n = 0

    def walk(block):
        nonlocal n
        uses, defs = {}, {}
        for it in block.items:
            if isinstance(it, (Loop, If)):
                walk(it.body)
                continue
            for v in it.srcs:
                uses[v.id] = uses.get(v.id, 0) + 1
            if it.dst is not None:
                defs[it.dst.id] = it
        dead = set()

        def single(v, kinds):
            d = defs.get(v.id)
            if d is None or d.kind not in kinds or id(d) in dead:
                return None
            # a doubling add(x, x) reads v twice
            return d if uses.get(v.id) == (2 if it.srcs[0].id == it.srcs[1].id else 1) else None

        for it in block.items:
            if isinstance(it, (Loop, If)) or it.kind != "add":
                continue
            a, b = it.srcs
            if a.id == b.id:                        # a doubling
                d = single(a, ("add", "shl"))
                if d is not None and (d.kind == "shl" or d.srcs[0].id == d.srcs[1].id):
                    sh = d.imm if d.kind == "shl" else 1
                    it.kind, it.srcs, it.imm = "shl", [d.srcs[0]], sh + 1
                    dead.add(id(d))
                    n += 1
                continue
            for j, v in enumerate((a, b)):
                other = it.srcs[1 - j]
                d = single(v, ("add", "shl"))
                if d is None:
                    continue
                if d.kind == "shl" or d.srcs[0].id == d.srcs[1].id:
                    sh = d.imm if d.kind == "shl" else 1
                    it.kind, it.srcs, it.imm = "shladd", [d.srcs[0], other], sh
                else:
                    it.kind, it.srcs = "add3", [d.srcs[0], d.srcs[1], other]
                dead.add(id(d))
                n += 1
                break
        block.items = [it for it in block.items if id(it) not in dead]

    walk(prog.root)
    return n


def check_scopes(prog):
    """Only named variables cross into loop / branch bodies: every Val used in
    a body is defined in that same body (the allocator relies on it)."""
    # simpler exact rule: track the defining block of each value
    owner = {}

    def mark(block):
        for it in block.items:
            if isinstance(it, (Loop, If)):
                mark(it.body)
            elif it.dst is not None:
                owner[it.dst.id] = id(block)
                if it.dst2 is not None:
                    owner[it.dst2.id] = id(block)

    def check(block):
        for it in block.items:
            if isinstance(it, (Loop, If)):
                check(it.body)
            else:
                for v in it.srcs:
                    assert owner[v.id] == id(block), "%r uses v%d defined in another block" % (it, v.id)
    mark(prog.root)
    check(prog.root)


class _Ctx:
    def __init__(self, prog, node):
        self.prog, self.node = prog, node

    def __enter__(self):
        self.prog.cur.items.append(self.node)
        self.prog.stack.append(self.prog.cur)
        self.prog.cur = self.node.body
        return self.node

    def __exit__(self, *exc):
        self.prog.cur = self.prog.stack.pop()
        return False


# ======================= exact evaluation =======================
class Stats:
    def __init__(self):
        self.counts = {}

    def bump(self, k, n=1):
        self.counts[k] = self.counts.get(k, 0) + n


def _check(limbs, u, what, half=False, vb=None):
    assert all(0 <= x <= u * MASK for x in limbs), "%s: limb bound u=%d violated" % (what, u)
    vb = u if vb is None else vb
    assert half or val_of(limbs) < vb * 2 * Q, "%s: value bound vb=%d violated" % (what, vb)


def wide_product(pairs):
    """normalized 28 limbs of sum a*b (column accumulation, carries folded)"""
    cols = [0] * (2 * NL)
    for a, b in pairs:
        for i in range(NL):
            for j in range(NL):
                cols[i + j] += a[i] * b[j]
    out, acc = [], 0
    for k in range(2 * NL - 1):
        acc += cols[k]
        assert acc < (1 << 64), "wide column %d overflows" % k
        out.append(acc & MASK)
        acc >>= LB
    assert acc <= MASK
    out.append(acc)
    return tuple(out[:NL]), tuple(out[NL:])


def wide_normalize(lo, hi):
    w = val_of(lo) + (val_of(hi) << (LB * NL))
    assert w < (1 << (LB * (2 * NL - 1) + LB)), "wide value exceeds 28 limbs"
    ls = [(w >> (LB * i)) & MASK for i in range(2 * NL - 1)] + [w >> (LB * (2 * NL - 1))]
    assert ls[-1] <= MASK
    return tuple(ls[:NL]), tuple(ls[NL:])


def mont_reduce_wide(lo, hi):
    """exact result of the emitted column reduction of lo + hi 2^392"""
    w = val_of(lo) + (val_of(hi) << (LB * NL))
    m = (-w * pow(Q, -1, R)) % R
    t = w + m * Q
    ml = gen_fl.limbs(m)
    acc = 0
    for k in range(2 * NL - 1):
        acc += (lo[k] if k < NL else hi[k - NL])
        acc += sum(ml[i] * QL[k - i] for i in range(max(0, k - NL + 1), min(k, NL - 1) + 1))
        assert acc < (1 << 64) - (1 << 36), "wred column %d overflows" % k
        acc >>= LB
    out = t // R
    assert out < (1 << 388), "wred output too large"
    return tuple(gen_fl.limbs(out))


def mont_sop(pairs):
    """exact result of the column-accumulator Montgomery product of sum a*b"""
    # column sums must fit the 64-bit accumulator (the static bound proves it;
    # check the concrete columns too)
    cols = [0] * (2 * NL)
    for a, b in pairs:
        for i in range(NL):
            for j in range(NL):
                cols[i + j] += a[i] * b[j]
    s = sum(int(a_) * int(b_) for a, b in pairs for a_, b_ in [(val_of(a), val_of(b))])
    m = (-s * pow(Q, -1, R)) % R
    t = s + m * Q
    assert t % R == 0
    ml = gen_fl.limbs(m)
    for k in range(2 * NL - 1):
        mq = sum(ml[i] * QL[k - i] for i in range(max(0, k - NL + 1), min(k, NL - 1) + 1))
        assert cols[k] + mq < (1 << 64) - (1 << 36), "column %d overflows" % k
    out = t // R
    assert out < R
    return tuple(gen_fl.limbs(out))


def val_of_signed(limbs):
    return sum(int(x) << (28 * i) for i, x in enumerate(limbs))


def mont_sop_signed(a, b):
    """exact limbs of emit_sop(signed=True): (s + m q) / R + q for s = a b with
    b's limbs signed, m = -s q^-1 mod R (the digits the leaf takes) plus R from
    the last digit's 2^28 -- every column of the signed 64-bit accumulator checked"""
    cols = [0] * (2 * NL)
    for i in range(NL):
        for j in range(NL):
            cols[i + j] += a[i] * b[j]
    s = val_of(a) * val_of_signed(b)
    m = (-s * pow(Q, -1, R)) % R
    ml = gen_fl.limbs(m)
    ml[NL - 1] += 1 << 28
    t = s + (m + R) * Q
    assert t % R == 0
    acc = 0
    for k in range(2 * NL - 1):
        acc += cols[k] + sum(ml[i] * QL[k - i] for i in range(max(0, k - NL + 1), min(k, NL - 1) + 1))
        assert -(1 << 63) <= acc < (1 << 63), "signed column %d overflows" % k
        acc >>= 28
    out = t // R
    assert 0 <= out < R
    return tuple(gen_fl.limbs(out))


def norm_limbs(x):
    """the emitted carry pass: limbs 0..12 below 2^28, the value unchanged"""
    r, c = [], 0
    for i in range(NL - 1):
        acc = x[i] + c
        assert acc < (1 << 32)
        r.append(acc & MASK)
        c = acc >> 28
    acc = x[NL - 1] + c
    assert acc < (1 << 32)
    r.append(acc)
    return tuple(r)


def red_limbs(x):
    p1 = x[12] * KQ
    p2 = x[13] * KQ
    k = (p2 + (p1 >> 28)) >> 36
    r = []
    acc = 0
    for i in range(NL - 1):
        acc += x[i] - k * QL[i]
        r.append(acc & MASK)
        acc >>= 28
    acc += x[13] - k * QL[13]
    assert 0 <= acc < (1 << 32)
    r.append(acc)
    return tuple(r)


# ---- the in-kernel binary GCD (emit.Emitter.emit_binv), limb-exact ----
# T. Pornin, "Optimized Binary GCD for Modular Inversion" (eprint 2020/972),
# Algorithm 2 with k - 1 = 28: BINV_OUTER outer steps of 28 inner steps on
# 58-bit approximations (the low 28 bits = limb 0, the top 30 bits of
# max(len a, len b, 58)); the update (u, v) <- (u f + v g) / 2^28 is one
# Montgomery digit, so u, v stay signed 14-limb integers below (t + 1) q in
# magnitude and are never reduced inside the loop.  28 x 28 = 784 >= 2 * 381 - 1.
BINV_OUTER = 28
BINV_PAD = 32          # v + 32 q >= 0 before the final product
BINV_C = pow(2, 3 * LB * NL, Q)       # R'^3: (y^-1) R'^3 / R' = a^-1 R' for y = a R'


def binv_core(y):
    """y (0 <= y < q) -> the signed integer v the emitted loop leaves (v = y^-1
    mod q, or 0 for y = 0), following the emitted limb arithmetic exactly"""
    A, B, U, W = y, Q, 1, 0
    m28 = MASK
    for _ in range(BINV_OUTER):
        n = max((A | B).bit_length(), 58)
        p = n - 30
        xa = (((A >> p) & ((1 << 30) - 1)) << 28) | (A & m28)
        xb = (((B >> p) & ((1 << 30) - 1)) << 28) | (B & m28)
        f0, g0, f1, g1 = 1, 0, 0, 1
        for _ in range(28):
            odd = xa & 1
            sw = odd and xa < xb
            if sw:
                xa, xb, f0, f1, g0, g1 = xb, xa, f1, f0, g1, g0
            if odd:
                xa, f0, g0 = xa - xb, f0 - f1, g0 - g1
            xa >>= 1
            f1, g1 = 2 * f1, 2 * g1
        na, nb = A * f0 + B * g0, A * f1 + B * g1
        assert na % (1 << 28) == 0 and nb % (1 << 28) == 0
        na >>= 28
        nb >>= 28
        if na < 0:
            na, f0, g0 = -na, -f0, -g0
        if nb < 0:
            nb, f1, g1 = -nb, -f1, -g1
        tu, tw = U * f0 + W * g0, U * f1 + W * g1
        ku = (tu * QINV28) & m28
        kw = (tw * QINV28) & m28
        tu, tw = tu + ku * Q, tw + kw * Q
        assert tu % (1 << 28) == 0 and tw % (1 << 28) == 0
        A, B, U, W = na, nb, tu >> 28, tw >> 28
    assert A == 0 and B in (1, Q), "binary GCD did not converge"
    return W


def binv_limbs(x):
    """limbs the emitted binv leaves for input limbs x: red, canonical y,
    the loop, v + 32 q normalized, times R'^3 (one Montgomery product)"""
    r = red_limbs(x)
    y = val_of(r)
    y = y - Q if y >= Q else y
    w = binv_core(y) + BINV_PAD * Q
    assert 0 <= w < (1 << 387)
    return mont_sop([(tuple(gen_fl.limbs(w)), tuple(gen_fl.limbs(BINV_C)))])


def evaluate(prog, inputs, stats=None, trace=None):
    """inputs: dict slot -> canonical ABI integer (R = 2^384 Montgomery value,
    i.e. the integer held in the record).  Returns dict slot -> output integer.
    Two-lane programs (prog.lanes == 2) run both lanes of a pair in lockstep;
    their load/store slots are (lane 0 slot, lane 1 slot) pairs."""
    L = prog.lanes
    env = {}
    vars_ = {}
    outs = {}
    counters = {}
    st = stats or Stats()

    def run(block):
        for it in block.items:
            if isinstance(it, Loop):
                for i in range(it.trips - 1, -1, -1):
                    counters[id(it)] = i
                    run(it.body)
            elif isinstance(it, If):
                if (it.mask >> counters[id(it.loop)]) & 1:
                    run(it.body)
            else:
                step(it)

    def lane_op(k, op, s):
        if k == "sop":
            return mont_sop(list(zip(s[0::2], s[1::2])))
        if k == "sqr":
            return mont_sop([(s[0], s[0])])
        if k == "ssop":
            return mont_sop_signed(s[0], s[1])
        if k == "add":
            return tuple(a + b for a, b in zip(*s))
        if k == "add3":
            return tuple(a + b + c for a, b, c in zip(*s))
        if k == "shladd":
            return tuple((a << op.imm) + b for a, b in zip(*s))
        if k == "shl":
            return tuple(a << op.imm for a in s[0])
        if k == "sub":
            c = SUBC[op.imm]
            return tuple(a + ci - b for a, ci, b in zip(s[0], c, s[1]))
        if k == "neg":
            c = SUBC[op.imm]
            return tuple(ci - b for ci, b in zip(c, s[0]))
        if k == "red":
            return red_limbs(s[0])
        if k == "norm":
            return norm_limbs(s[0])
        if k == "csub":
            return tuple(a + ci - b for a, ci, b in zip(s[0], op.imm, s[1]))
        if k == "wred":
            return mont_reduce_wide(s[0], s[1])
        if k == "inv":
            v = val_of(s[0]) % Q
            return tuple(gen_fl.limbs(R * R * pow(v, -1, Q) % Q if v else 0))
        if k == "binv":
            return binv_limbs(s[0])
        if k == "selz":
            nt = op.imm
            return s[nt] if all(val_of(t) % Q == 0 for t in s[:nt]) else s[nt + 1]
        raise ValueError(k)

    def step(op):
        k = op.kind
        s = [env[v.id] for v in op.srcs]      # per source: list over lanes
        st.bump(k)
        if k == "sop":
            st.bump("sop%d" % (len(op.srcs) // 2))
        if k == "const":
            r = [op.imm] * L
        elif k == "getvar":
            r = vars_[op.imm]
        elif k == "setvar":
            vars_[op.imm] = s[0]
            return
        elif k == "arg":
            r = [tuple(inputs[op.imm])] * L
        elif k == "ret":
            outs[op.imm] = s[0][0]
            return
        elif k == "load_raw":
            slots = op.imm if isinstance(op.imm, tuple) else (op.imm,) * L
            r = [tuple(gen_fl.limbs(inputs[slots[ln]])) for ln in range(L)]
        elif k == "tload":
            r = [tuple(inputs["lines"][counters.get("line", 0)][op.imm])] * L
        elif k == "tnext":
            counters["line"] = counters.get("line", 0) + 1
            return
        elif k == "store_raw":
            slots = op.imm if isinstance(op.imm, tuple) else (op.imm,) * L
            for ln in range(L):
                v = val_of(s[0][ln])
                assert v < 2 * Q
                outs[slots[ln]] = v % Q
            return
        elif k == "swap":
            r = [s[0][1 - ln] for ln in range(L)]
        elif k == "sel":
            r = [s[ln][ln] for ln in range(L)]
        elif k == "bcast":
            r = [s[0][op.imm] for ln in range(L)]
        elif k == "pairz":
            c = SUBC[op.imm]
            r = [tuple(ci - b for ci, b in zip(c, s[0][1])), s[0][1]]
        elif k == "pdiff":
            r = [tuple(x - y for x, y in zip(s[0][0], s[0][1])), s[0][0]]
            for ln in range(L):
                assert all(-op.dst.u * MASK < x <= op.dst.u * MASK for x in r[ln]), "pdiff limb bound"
                assert abs(val_of_signed(r[ln])) < op.dst.vb * 2 * Q, "pdiff value bound"
            env[op.dst.id] = r
            if trace is not None:
                trace.append((op.dst.id, tuple(r), op))
            return
        elif k == "dppadd":
            r = [tuple(x + y for x, y in zip(s[0][op.imm[ln]], s[1][ln])) for ln in range(L)]
        elif k in ("wsop", "wnorm"):
            if k == "wsop":
                st.bump("wsop%d" % (len(op.srcs) // 2))
                lh = [wide_product(list(zip([x[ln] for x in s][0::2], [x[ln] for x in s][1::2])))
                      for ln in range(L)]
            else:
                lh = [wide_normalize(s[0][ln], s[1][ln]) for ln in range(L)]
            for ln in range(L):
                _check(lh[ln][0], op.dst.u, repr(op), True)
                _check(lh[ln][1], op.dst2.u, repr(op), True)
            env[op.dst.id] = [x[0] for x in lh]
            env[op.dst2.id] = [x[1] for x in lh]
            if trace is not None:
                trace.append((op.dst.id, lh[0][0] if L == 1 else tuple(x[0] for x in lh), op))
                trace.append((op.dst2.id, lh[0][1] if L == 1 else tuple(x[1] for x in lh), op))
            return
        else:
            r = [lane_op(k, op, [x[ln] for x in s]) for ln in range(L)]
        for ln in range(L):
            _check(r[ln], op.dst.u, repr(op), op.dst.half, op.dst.vb)
        env[op.dst.id] = r
        if trace is not None:
            trace.append((op.dst.id, r[0] if L == 1 else tuple(r), op))

    run(prog.root)
    return outs
