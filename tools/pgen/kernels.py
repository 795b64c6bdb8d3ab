"""The two generated kernels as DSL programs.

  miller_loop   inputs  0 px, 1 py, 2 qx.c0, 3 qx.c1, 4 qy.c0, 5 qy.c1
                outputs 0..11 the Fq12 coordinates (ABI order)
                = Bls12::miller_loop([(P, Q.prepare())]) (mod.rs:40-102)
  final_exp     inputs / outputs 0..11 Fq12 coordinates
                = Bls12::final_exponentiation (mod.rs:104-160)

Infinity inputs (miller loop -> one) and f == 0 (final exp -> None) are
lane selects done by the emitted prologue/epilogue, outside the DSL.
"""
import os

from dsl import Prog
from tower import Tower, TowerLazy, TowerLazySq, X_ABS, declare12, get12, set12  # noqa: F401
from tower2 import Tower2

ML_MASK = (X_ABS >> 1) & ((1 << 62) - 1)  # bits 61..0 below the leading one of |x| >> 1


def _norm(lanes):
    """carry-normalize instead of reducing where value bounds allow (dsl.VB_PROD);
    round 5: lane-pair kernels too (-1 % instructions; PGEN_NORM2=0 keeps the full
    reduction there); PGEN_NORM=0: the full reduction everywhere, A/B"""
    if lanes == 2 and os.environ.get("PGEN_NORM2", "1") != "1":
        return False
    return os.environ.get("PGEN_NORM", "1") == "1"


def doubling_step(T, r):
    """mod.rs:176-245 (Algorithm 26, eprint 2010/354)"""
    x, y, z = r
    tmp0 = T.sqr2(x)
    tmp1 = T.sqr2(y)
    tmp2 = T.sqr2(tmp1)
    tmp3 = T.red2(T.dbl2(T.sub2(T.sqr2(T.add2(tmp1, x)), T.add2(tmp0, tmp2))))
    tmp4 = T.red2(T.add2(T.dbl2(tmp0), tmp0))
    tmp6 = T.add2(x, tmp4)
    tmp5 = T.sqr2(tmp4)
    zsq = T.sqr2(z)
    nx = T.red2(T.sub2(tmp5, T.dbl2(tmp3)))
    nz = T.red2(T.sub2(T.sqr2(T.add2(z, y)), T.add2(tmp1, zsq)))
    ny = T.red2(T.sub2(T.mul2(T.sub2(tmp3, nx), tmp4), T.dbl2(T.dbl2(T.dbl2(tmp2)))))
    c1 = T.red2(T.neg2(T.dbl2(T.mul2(tmp4, zsq))))
    c2 = T.red2(T.sub2(T.sub2(T.sqr2(tmp6), T.add2(tmp0, tmp5)), T.dbl2(T.dbl2(tmp1))))
    c0 = T.red2(T.dbl2(T.mul2(nz, zsq)))
    return (c0, c1, c2), (nx, ny, nz)


def addition_step(T, r, qx, qy):
    """mod.rs:247-333 (Algorithm 27, eprint 2010/354)"""
    rx, ry, rz = r
    zsq = T.sqr2(rz)
    ysq = T.sqr2(qy)
    t0 = T.mul2(zsq, qx)
    t1 = T.mul2(T.sub2(T.sqr2(T.add2(qy, rz)), T.add2(ysq, zsq)), zsq)
    t2 = T.red2(T.sub2(t0, rx))
    t3 = T.sqr2(t2)
    t4 = T.dbl2(T.dbl2(t3))
    t5 = T.mul2(t4, t2)
    t6 = T.red2(T.sub2(t1, T.dbl2(ry)))
    t9 = T.mul2(t6, qx)
    t7 = T.mul2(t4, rx)
    nx = T.red2(T.sub2(T.sqr2(t6), T.add2(t5, T.dbl2(t7))))
    nz = T.red2(T.sub2(T.sqr2(T.add2(rz, t2)), T.add2(zsq, t3)))
    t8 = T.mul2(T.sub2(t7, nx), t6)
    ny = T.red2(T.sub2(t8, T.dbl2(T.mul2(ry, t5))))
    t10 = T.sub2(T.sqr2(T.add2(qy, nz)), T.add2(ysq, T.sqr2(nz)))
    c2 = T.red2(T.sub2(T.dbl2(t9), t10))
    c0 = T.red2(T.dbl2(nz))
    c1 = T.red2(T.dbl2(T.neg2(t6)))
    return (c0, c1, c2), (nx, ny, nz)


def doubling_step_h(T, r):
    """doubling with its tangent line in homogeneous coordinates (x = X/Z,
    y = Y/Z) on E': y^2 = x^3 + b', b' = 4 (1 + u) (Costello-Lange-Naehrig,
    eprint 2009/615, scaled by 4 to avoid halvings): 3 M + 6 S against
    doubling_step's 3 M + 8 S.  The line is the reference's scaled by an Fq2
    factor (Z^2 / 2 Z_J^6): c0 = 2 Y Z (y_P), c1 = -3 X^2 (x_P), c2 = Y^2 - 3 b' Z^2
    -- equal after the final exponentiation, not as a Miller value
    (pairing-only kernels)"""
    x, y, z = r
    B = T.sqr2(y)
    C = T.sqr2(z)
    xc = T.red2(T.xi(C))
    E = T.red2(T.dbl2(T.dbl2(T.add2(T.dbl2(xc), xc))))          # 12 (1 + u) Z^2 = 3 b' Z^2
    H = T.red2(T.sub2(T.sqr2(T.add2(y, z)), T.add2(B, C)))        # 2 Y Z
    X2 = T.sqr2(x)
    E3 = T.red2(T.add2(T.dbl2(E), E))
    nx = T.red2(T.dbl2(T.mul2(T.mul2(x, y), T.red2(T.sub2(B, E3)))))   # 2 X Y (Y^2 - 9 b' Z^2)
    ee = T.sqr2(E)
    e12 = T.dbl2(T.dbl2(T.add2(T.dbl2(ee), ee)))
    ny = T.red2(T.sub2(T.sqr2(T.red2(T.add2(B, E3))), e12))   # (Y^2 + 9 b' Z^2)^2 - 108 b'^2 Z^4
    nz = T.red2(T.dbl2(T.dbl2(T.mul2(B, H))))                 # 8 Y^3 Z
    c1 = T.red2(T.neg2(T.add2(T.dbl2(X2), X2)))
    c2 = T.red2(T.sub2(B, E))
    return (H, c1, c2), (nx, ny, nz)


def addition_step_h(T, r, qx, qy):
    """mixed addition R + Q (R homogeneous, Q affine) with the line through
    them: theta = Y1 - y2 Z1, lambda = X1 - x2 Z1; the line lambda y_P -
    theta x_P + (theta x2 - lambda y2) is the reference's scaled by an Fq2
    factor (pairing-only kernels)"""
    X1, Y1, Z1 = r
    th = T.red2(T.sub2(Y1, T.mul2(qy, Z1)))
    la = T.red2(T.sub2(X1, T.mul2(qx, Z1)))
    cc = T.sqr2(th)
    d = T.sqr2(la)
    e = T.mul2(la, d)
    f = T.mul2(Z1, cc)
    g = T.mul2(X1, d)
    h = T.red2(T.sub2(T.add2(e, f), T.dbl2(g)))
    nx = T.mul2(la, h)
    ny = T.red2(T.sub2(T.mul2(th, T.red2(T.sub2(g, h))), T.mul2(Y1, e)))
    nz = T.mul2(Z1, e)
    c1 = T.red2(T.neg2(th))
    c2 = T.red2(T.sub2(T.mul2(th, qx), T.mul2(la, qy)))
    return (la, c1, c2), (nx, ny, nz)


def ell(T, f, c, px, py):
    """mod.rs:57-69: f.mul_by_014(c2, c1 * P.x, c0 * P.y)"""
    return T.mul_by_014(f, c[2], T.mul_fq(c[1], px), T.mul_fq(c[0], py))


ML_HOMES = {"px": "L", "py": "L", "qx0": "M", "qx1": "M", "qy0": "M", "qy1": "M",
            "rx0": "A", "rx1": "A", "ry0": "A", "ry1": "A", "rz0": "A", "rz1": "A", "f": "A"}
# the Fq12 variable names f<i>_<c> carry the home of "f"
# lane pairs (no AGPRs, 5 LDS slots): f -- read by every line and square -- in
# five of the LDS slots, P's packed coordinates and the G2 point (read once per
# step) in the workspace: half the workspace traffic of the AGPR-first homes
# (1119 -> 545 loads, 657 -> 341 stores per lane; PGEN_ML2_HOMES=0: the old homes)
ML2_HOMES = {"f": "LLLLLLLLLLMM", "px": "M", "rx0": "M", "ry0": "M", "rz0": "M"}


def miller_loop_prog(homes=None, lanes=1, lazy=False, pairing_only=False):
    """pairing_only: the G2 steps in homogeneous coordinates with their own
    line scaling (doubling_step_h / addition_step_h): f differs from the
    reference's Miller value by an Fq2 factor, which the final exponentiation
    removes ((q^12 - 1) / r is a multiple of q^2 - 1) -- for e(P, Q) only"""
    base = dict(ML_HOMES, **ML2_HOMES) if lanes == 2 and os.environ.get("PGEN_ML2_HOMES", "1") == "1" else ML_HOMES
    homes = dict(base, **(homes or {}))
    name = ("miller_loop" if lanes == 1 else "miller_loop2") + ("p" if pairing_only else "")
    p = Prog(name, lanes, use_norm=_norm(lanes))
    dbl, add = (doubling_step_h, addition_step_h) if pairing_only else (doubling_step, addition_step)
    T = (TowerLazy(p) if lazy else Tower(p)) if lanes == 1 else Tower2(p)
    V = _Vars(p, lanes)
    for n in ("px", "py"):
        p.var(n, 1, homes.get(n))
    if lanes == 1:
        p.set("px", p.load(0))
        p.set("py", p.load(1))
    else:
        p.set("px", p.load(0, 1))    # lane 0: px, lane 1: py
    for n in ("qx0", "qx1", "qy0", "qy1", "rx0", "rx1", "ry0", "ry1", "rz0", "rz1"):
        p.var(n, 1, homes.get(n))
    V.set2("qx", (p.load(2), p.load(3)) if lanes == 1 else p.load(2, 3))
    V.set2("qy", (p.load(4), p.load(5)) if lanes == 1 else p.load(4, 5))
    V.declare12("f", homes.get("f"))
    zero = T.const2((0, 0))
    V.set2("rx", V.get2("qx"))
    V.set2("ry", V.get2("qy"))
    V.set2("rz", T.one2())
    V.set12("f", ((T.one2(), zero, zero), (zero, zero, zero)))

    def line(step):
        r = tuple(V.get2(n) for n in ("rx", "ry", "rz"))
        if step == "dbl":
            c, r = dbl(T, r)
        else:
            c, r = add(T, r, V.get2("qx"), V.get2("qy"))
        for n, v in zip(("rx", "ry", "rz"), r):
            V.set2(n, v)
        if lanes == 1:
            px, py = p.get("px"), p.get("py")
        else:   # replicate P's coordinates from the packed (px | py) slot
            pk = p.get("px")
            px, py = p.bcast(pk, 0), p.bcast(pk, 1)
        V.set12("f", ell(T, V.get12("f"), c, px, py))

    with p.loop(62) as L:
        line("dbl")
        with p.if_bit(ML_MASK, L):
            line("add")
        V.set12("f", T.sqr12(V.get12("f")))
    line("dbl")
    V.store12(T.conj12(V.get12("f")))
    return p


def miller_loop_prepared_prog():
    """Bls12::miller_loop over (G1Affine_i, G2Prepared_i) pairs -- the
    north-star call shape (mod.rs:40-102 with each pair's own prepared record):
    miller_loop_shared_prog with the lines read from this lane's G2Prepared
    record (kcfg.MillerLoopPreparedCfg) in the ABI form, all six values raw;
    c2 takes its lazy form by one product each (prepared_table_lines)"""
    return miller_loop_shared_prog(per_lane=True)


def prepared_table_lines(coeffs):
    """the values tload gives miller_loop_prepared_prog: raw limbs of the six
    ABI integers of every line (the record as written by k_g2_prepare)"""
    import gen_fl
    return [[tuple(gen_fl.limbs(x)) for x in line] for line in coeffs]


def miller_loop_shared_prog(per_lane=False):
    """Bls12::miller_loop([(P_i, Q)]) for a batch of P_i and ONE prepared Q
    (lib.rs:88-96 with the same &G2Prepared in every pair; mod.rs:40-102).
    No G2 arithmetic: the line coefficients come from the kernel's line table
    (kcfg.MillerLoopSharedCfg), six values per line as written by
    k_shared_line_table (kernels_pairing.hip):
      0, 1  c0 = (c0.c0, c0.c1)  raw limbs of the ABI integer (x R, R = 2^384)
      2, 3  c1                   likewise
      4, 5  c2                   lazy form (x R', R' = 2^392)
    and P's coordinates are loaded scaled by 2^408 (x R' (R'/R)), so that
    mul(raw c, kx) = c P.x R' -- the ABI -> lazy conversion of c0 and c1 rides
    on the products ell needs anyway (mod.rs:57-69; pairing_fl.h ell_fl).
      inputs 0 px, 1 py (this lane's G1Affine); outputs 0..11 (Fq12)"""
    p = Prog("miller_loop_prepared" if per_lane else "miller_loop_shared", 1, use_norm=_norm(1))
    T = Tower(p)
    V = _Vars(p, 1)
    for n in ("kx", "ky"):
        p.var(n, 1, "A")
    p.set("kx", p.load_scaled(0, 1 << 408))
    p.set("ky", p.load_scaled(1, 1 << 408))
    V.declare12("f", os.environ.get("PGEN_MLS_F_HOME", "A"))
    zero = T.const2((0, 0))
    V.set12("f", ((T.one2(), zero, zero), (zero, zero, zero)))

    def line():
        c = [p.tload(j) for j in range(6)]
        if not per_lane:
            p.tnext()
        if per_lane:
            # c2 raw from the record (c2 R): its lazy form c2 R' = raw 2^8 mod q,
            # two rounds of x16 (limbs < 2^32) and a reduction -- in place of a
            # product by 2^400 (R'^2 / R)
            for j in (4, 5):
                for _ in range(2):
                    for _ in range(4):
                        c[j] = p.add(c[j], c[j])
                    c[j] = p.red(c[j])
        kx, ky = p.get("kx"), p.get("ky")
        a = (p.mul(c[0], ky), p.mul(c[1], ky))     # c0 * P.y
        b = (p.mul(c[2], kx), p.mul(c[3], kx))     # c1 * P.x
        if per_lane:
            # every value of the line is in registers: the next line's copy into
            # the LDS buffer (kcfg.MillerLoopPreparedCfg) lands under mul_by_014
            p.tnext()
        V.set12("f", T.mul_by_014(V.get12("f"), (c[4], c[5]), b, a))

    with p.loop(62) as L:
        line()
        with p.if_bit(ML_MASK, L):
            line()
        V.set12("f", T.sqr12(V.get12("f")))
    line()
    V.store12(T.conj12(V.get12("f")))
    return p


def shared_table_lines(coeffs):
    """the line table values of miller_loop_shared_prog for 68 lines of six
    ABI integers (c0.c0, c0.c1, c1.c0, c1.c1, c2.c0, c2.c1; x R, canonical):
    raw limbs for c0 and c1, the lazy form mul(raw, 2^400) for c2 -- exactly
    the limbs k_shared_line_table (kernels_pairing.hip) writes"""
    import gen_fl
    from dsl import mont_sop, Q
    to = tuple(gen_fl.limbs(pow(2, 400, Q)))
    out = []
    for line in coeffs:
        raw = [tuple(gen_fl.limbs(x)) for x in line]
        out.append(raw[:4] + [mont_sop([(r, to)]) for r in raw[4:]])
    return out


def shared_table_u64(lines, infinity):
    """the table as u64 words (kcfg.MillerLoopSharedCfg layout): u32 word 0 the
    infinity flag, lines from byte 64, 14 u32 limbs per value"""
    words32 = [1 if infinity else 0] + [0] * 15
    for line in lines:
        for v in line:
            words32 += list(v)
    if len(words32) % 2:
        words32.append(0)
    return [words32[2 * k] | (words32[2 * k + 1] << 32) for k in range(len(words32) // 2)]


class _Vars:
    """Fq2 / Fq12 state variables: a one-lane Fq2 is two variables (c0, c1),
    a distributed Fq2 one variable per lane (named <n>0; <n>1 unused)."""

    def __init__(self, p, lanes):
        self.p, self.lanes = p, lanes

    def get2(self, n):
        p = self.p
        return (p.get(n + "0"), p.get(n + "1")) if self.lanes == 1 else p.get(n + "0")

    def set2(self, n, v):
        p = self.p
        if self.lanes == 1:
            p.set(n + "0", v[0])
            p.set(n + "1", v[1])
        else:
            p.set(n + "0", v)

    def declare12(self, prefix, home=None):
        """home: one storage tier for all 12 coordinates, or a 12-character string
        of tiers per coordinate (e.g. "AAAAAAMMMMMM")"""
        for i in range(6):
            for c in (0, 1):
                h = home[2 * i + c] if home is not None and len(home) == 12 else home
                self.p.var("%s%d_%d" % (prefix, i, c), 1, h)

    def get12(self, prefix):
        xs = [self.get2("%s%d_" % (prefix, i)) for i in range(6)]
        return ((xs[0], xs[1], xs[2]), (xs[3], xs[4], xs[5]))

    def set12(self, prefix, f):
        for i, v in enumerate([x for c6 in f for x in c6]):
            self.set2("%s%d_" % (prefix, i), v)

    def store12(self, f):
        """ABI order: coordinate (2i + c) of Fq2 number i"""
        for i, v in enumerate([x for c6 in f for x in c6]):
            if self.lanes == 1:
                self.p.store(2 * i, v[0])
                self.p.store(2 * i + 1, v[1])
            else:
                self.p.store(2 * i, v, 2 * i + 1)

    def load12(self):
        p = self.p
        if self.lanes == 1:
            xs = [(p.load(2 * i), p.load(2 * i + 1)) for i in range(6)]
        else:
            xs = [p.load(2 * i, 2 * i + 1) for i in range(6)]
        return ((xs[0], xs[1], xs[2]), (xs[3], xs[4], xs[5]))


def exp_by_x(p, T, V, f, x, tag):
    """exp_by_x (mod.rs:116-121): f^|x| by square-and-multiply (lib.rs:306-324)
    with cyclotomic squarings, then conjugation (x < 0)"""
    base, res = "eb%s_" % tag, "er%s_" % tag
    # the base f: 8 coordinates in AGPRs, 4 in the HBM workspace (FE 11.37 -> 11.11 ms
    # against all 12 in HBM, profiles/r02_eb_home_ab.txt)
    V.declare12(base, os.environ.get("PGEN_EB_HOME", "AAAAAAAAMMMM"))
    V.declare12(res, os.environ.get("PGEN_ER_HOME", "A"))
    V.set12(base, f)
    V.set12(res, f)
    top = x.bit_length() - 1
    with p.loop(top) as L:
        V.set12(res, T.cyc_sqr(V.get12(res)))
        with p.if_bit(x & ((1 << top) - 1), L):
            V.set12(res, T.mul12(V.get12(res), V.get12(base)))
    return T.conj12(V.get12(res))


def exp_by_x_karabina(p, T, V, xv, L, first_skip, tag="k"):
    """exp_by_x (mod.rs:116-121) in place on the Fq12 variable `xv`, as
    f^|x| = prod f^(2^i) over the set bits i of |x| = 0xd201000000010000
    (16, 48, 57, 60, 62, 63), then conjugation (x < 0).  The powers up to
    bit 57 come from ONE run of compressed (Karabina) squarings, saved at bits
    16 and 48; those three are decompressed with one shared inversion
    (Tower.batch_inv2 -> the in-kernel binary GCD); the 6 squarings between the
    top bits run uncompressed (Granger-Scott) from f^(2^57), since another
    decompression would cost more than they do.  Inside the hard part's loop
    over its five calls (final_exp_prog): when bit `first_skip` of the loop
    counter L is set the first run is one squaring shorter, which is the
    exp_by_x(x >> 1) call (bits 15, 47, 56, 59, 61, 62)."""
    bits = [i for i in range(X_ABS.bit_length()) if (X_ABS >> i) & 1]
    res, top = "kr%s_" % tag, "kt%s_" % tag
    one = p.lanes == 1   # lane pairs: a distributed Fq2 is one variable (<n>0)
    # the compressed state's homes are those of the later GS state's first 4
    # Fq2 coordinates (the two never live at once)
    kn = ["%s%d_%d" % (top, j // 2, j % 2) for j in range(8)] if one else ["%s%d_0" % (top, i) for i in range(4)]
    for n in kn:
        p.var(n, 1, os.environ.get("PGEN_KC_HOME", "A"))
    (_, a1, a2), (b0, _, b2) = V.get12(xv)
    for n, v in zip(kn, [*a1, *a2, *b0, *b2] if one else [a1, a2, b0, b2]):
        p.set(n, v)

    def getg(names):
        g = [p.get(n) for n in names]
        return ((g[0], g[1]), (g[2], g[3]), (g[4], g[5]), (g[6], g[7])) if one else tuple(g)

    def flat(g4):
        return [c for x2 in g4 for c in x2] if one else list(g4)

    def ksqr_state():
        for n, v in zip(kn, flat(T.ksqr(getg(kn)))):
            p.set(n, v)

    saved, prev = [], 0
    for k, b in enumerate(bits[:3]):
        n = b - prev
        if k == 0:
            n -= 1
        with p.loop(n):
            ksqr_state()
        if k == 0:
            with p.if_bit(((1 << 8) - 1) & ~(1 << first_skip), L):
                ksqr_state()
        prev = b
        if k < 2:
            sn = ["ks%s%d_%d" % (tag, k, i) for i in range(len(kn))]
            for n in sn:
                p.var(n, 1, os.environ.get("PGEN_KS_HOME", "M"))
            for n, v in zip(sn, [p.get(m) for m in kn]):
                p.set(n, v)
            saved.append(sn)
    saved.append(kn)
    nds = [T.kdec_numden(getg(sn)) for sn in saved]
    idens = T.batch_inv2([nd[1] for nd in nds], tag)
    order = os.environ.get("PGEN_KDEC_ORDER", "1")   # "0": the round-3 order (A/B)
    fin = lambda k: T.kdec_finish(getg(saved[k]), nds[k][0], idens[k], nds[k][2])
    if order == "0":
        F = [fin(k) for k in range(3)]
    # top: the GS state reuses the 8 compressed-state homes (dead by now) plus
    # four more; res: 6 + 6 coordinates in AGPRs + the workspace
    V.declare12(res, os.environ.get("PGEN_KR_HOME", "AAAAAAMMMMMM"))
    for i in range(4, 6):
        for c in ((0, 1) if one else (0,)):
            p.var("%s%d_%d" % (top, i, c), 1, os.environ.get("PGEN_KT_HOME", "A"))
    if order == "0":
        V.set12(top, F[2])
        V.set12(res, T.mul12(T.mul12(F[0], F[1]), F[2]))
    else:
        # (default) finish the top state first, straight into its homes, then the two
        # snapshots one after the other into their product: 12 fewer M slots,
        # 15% fewer workspace moves, FE 9.29 -> 9.11 ms (profiles/r04_kdec_order.txt)
        V.set12(top, fin(2))
        V.set12(res, T.mul12(fin(0), fin(1)))
        V.set12(res, T.mul12(V.get12(res), V.get12(top)))
    # the top bits: squarings 1..6 above bit 57, multiply after squarings 3, 5, 6
    # (loop counter 5..0 -> bits 3, 1, 0 of the mask)
    assert [b - bits[2] for b in bits[3:]] == [3, 5, 6]
    with p.loop(6) as L2:
        V.set12(top, T.cyc_sqr(V.get12(top)))
        with p.if_bit(0b1011, L2):
            V.set12(res, T.mul12(V.get12(res), V.get12(top)))
    V.set12(xv, T.conj12(V.get12(res)))


def hard_part_loop(p, T, V, r):
    """mod.rs:125-156 with the five exp_by_x calls as ONE loop body (counter
    4..0 = calls a..e; the code between calls runs in branches on the counter),
    so the final exponentiation's code holds one copy of exp_by_x.  Returns y1.
        a: y1 = E(y0)                b: y2 = E'(y1)  (x >> 1)
           y1 = conj(y1 conj(r)) y2  c: y2 = E(y1)   d: y3 = E(y2)
           y1 = frob3(conj(conj(y1) ...)) ... (see below)    e: y2 = E(y3)"""
    H = os.environ.get("PGEN_HP_HOME", "M")
    for n in ("hr", "y0", "y1", "y2", "x"):
        V.declare12(n, H)
    V.set12("hr", r)
    y0 = T.cyc_sqr(r)
    V.set12("y0", y0)
    V.set12("x", y0)
    with p.loop(5) as L:
        exp_by_x_karabina(p, T, V, "x", L, first_skip=3)
        with p.if_bit(1 << 4, L):          # after a: y1 = E(y0)
            V.set12("y1", V.get12("x"))
        with p.if_bit(1 << 3, L):          # after b: y2 = E'(y1); y1 = conj(y1 conj(r)) y2
            y2 = V.get12("x")
            y1 = T.mul12(T.conj12(T.mul12(V.get12("y1"), T.conj12(V.get12("hr")))), y2)
            V.set12("y1", y1)
            V.set12("x", y1)
        with p.if_bit(1 << 2, L):          # after c: y2 = E(y1)
            V.set12("y2", V.get12("x"))
        with p.if_bit(1 << 1, L):          # after d: y3 = E(y2) (stays in x)
            y3 = V.get12("x")
            y1 = V.get12("y1")
            y1c = T.conj12(y1)
            y3 = T.mul12(y3, y1c)
            y1 = T.mul12(T.frob12(y1, 3), T.frob12(V.get12("y2"), 2))
            V.set12("y1", y1)
            V.set12("y2", y3)              # y2 holds y3 until the end
            V.set12("x", y3)
    # after e: x = E(y3); y3 is in y2
    y2 = T.mul12(T.mul12(V.get12("x"), V.get12("y0")), V.get12("hr"))
    y1 = T.mul12(V.get12("y1"), y2)
    return T.mul12(y1, T.frob12(V.get12("y2"), 1))


def hard_part_loop_folded(p, T, V, r):
    """mod.rs:125-156 as hard_part_loop, with every factor of the result folded
    into one accumulator `u` as soon as it exists, so at most two Fq12 values
    are parked across an exp_by_x (hard_part_loop parks up to four).  With
    E = exp_by_x (a homomorphism on the cyclotomic subgroup, conj = inverse):
      a: y1 = E(r^2)            b: y2 = E'(y1);  Y = conj(y1) r y2   (y1 of mod.rs:133-135)
      c: y2 = E(Y)              d: z = E(y2)  (mod.rs' y3 = z conj(Y))
      e: E(y3) = E(z) conj(y2)
    result = Y^(q^3) y2^(q^2) (z conj(Y))^q E(z) conj(y2) r^3
           = [Y^(q^3) conj(Y)^q r^3]_b [y2^(q^2) conj(y2)]_c [z^q]_d E(z)_e.
    u holds r until b, then the accumulated product; v holds y1 from a to b."""
    H = os.environ.get("PGEN_HP_HOME", "M")
    for n in ("u", "v", "x"):
        V.declare12(n, H)
    V.set12("u", r)
    V.set12("x", T.cyc_sqr(r))
    with p.loop(5) as L:
        exp_by_x_karabina(p, T, V, "x", L, first_skip=3)
        with p.if_bit(1 << 4, L):          # after a: y1 = E(r^2)
            V.set12("v", V.get12("x"))
        with p.if_bit(1 << 3, L):          # after b: Y = conj(y1 conj(r)) y2; u = Y^(q^3) conj(Y)^q r^3
            r_ = V.get12("u")
            y = T.mul12(T.conj12(T.mul12(V.get12("v"), T.conj12(r_))), V.get12("x"))
            V.set12("x", y)
            r3 = T.mul12(T.cyc_sqr(r_), r_)
            V.set12("u", T.mul12(T.mul12(T.frob12(y, 3), T.frob12(T.conj12(y), 1)), r3))
        with p.if_bit(1 << 2, L):          # after c: u *= y2^(q^2) conj(y2)
            y2 = V.get12("x")
            V.set12("u", T.mul12(V.get12("u"), T.mul12(T.frob12(y2, 2), T.conj12(y2))))
        with p.if_bit(1 << 1, L):          # after d: u *= z^q
            V.set12("u", T.mul12(V.get12("u"), T.frob12(V.get12("x"), 1)))
    return T.mul12(V.get12("u"), V.get12("x"))


def _karabina():
    return os.environ.get("PGEN_KARABINA", "1") == "1"


def final_exp_prog(lanes=1, lazy=False, tower_cls=None, split=None):
    """lazy: False (Tower), True (TowerLazy) or "sq" (TowerLazySq);
    tower_cls overrides the tower class (coop.py: inversion as one op).
    split (one lane): the final exponentiation in two kernels around a
    base-field inversion run elsewhere (binary GCD, bgcd.h) instead of the
    463-product Fermat chain -- "norm": load f, compute the Fq value that
    f^-1 needs inverted (fq12.rs:132-148 -> fq6.rs:250-301 -> fq2.rs:138-155)
    and store it as output slot 0; "inv": the whole final exponentiation with
    that value's inverse read from input slot 12"""
    p = Prog("final_exp" if lanes == 1 else "final_exp2", lanes,
             use_norm=_norm(lanes) and tower_cls is None)
    if tower_cls is not None:
        T = tower_cls(p)
    elif lanes == 2:
        T = Tower2(p)
    else:
        T = {False: Tower, True: TowerLazy, "sq": TowerLazySq}[lazy](p)
    V = _Vars(p, lanes)
    # one-lane programs invert in the kernel by binary GCD (emit.emit_binv) and
    # exponentiate by x with compressed squarings; PGEN_KARABINA=0: Fermat +
    # Granger-Scott (round 2)
    # lane pairs (round 5, PGEN_FE2_KARA=0: round 2's form for A/B): the same
    # Karabina squarings and in-kernel binary GCD (Tower2's kdec_numden / inv2)
    kara = ((lanes == 1 or os.environ.get("PGEN_FE2_KARA", "1") == "1") and tower_cls is None and split is None
            and _karabina())
    p.binv_ok = kara
    f = V.load12()
    if split is not None:
        assert lanes == 1 and split in ("norm", "inv")
        T.fe_split = split
    if split == "norm":
        from tower import NormStop
        try:
            T.inv12(f)
        except NormStop as stop:
            p.store(0, stop.args[0])
            return p
        raise AssertionError("inv12 did not reach the base-field inversion")
    # mod.rs:104-160
    f1 = T.conj12(f)
    f2 = T.inv12(f)
    r = T.mul12(f1, f2)
    f2 = r
    r = T.mul12(T.frob12(r, 2), f2)
    if kara:
        hp = hard_part_loop_folded if os.environ.get("PGEN_HP_FOLD", "0") == "1" else hard_part_loop
        V.store12(hp(p, T, V, r))
        return p
    x = X_ABS
    y0 = T.cyc_sqr(r)
    y1 = exp_by_x(p, T, V, y0, x, "a")
    y2 = exp_by_x(p, T, V, y1, x >> 1, "b")
    y3 = T.conj12(r)
    y1 = T.mul12(y1, y3)
    y1 = T.conj12(y1)
    y1 = T.mul12(y1, y2)
    y2 = exp_by_x(p, T, V, y1, x, "c")
    y3 = exp_by_x(p, T, V, y2, x, "d")
    y1 = T.conj12(y1)
    y3 = T.mul12(y3, y1)
    y1 = T.conj12(y1)
    y1 = T.frob12(y1, 3)
    y2 = T.frob12(y2, 2)
    y1 = T.mul12(y1, y2)
    y2 = exp_by_x(p, T, V, y3, x, "e")
    y2 = T.mul12(y2, y0)
    y2 = T.mul12(y2, r)
    y1 = T.mul12(y1, y2)
    y2 = T.frob12(y3, 1)
    y1 = T.mul12(y1, y2)
    V.store12(y1)
    return p
