"""The two generated kernels as DSL programs.

  miller_loop   inputs  0 px, 1 py, 2 qx.c0, 3 qx.c1, 4 qy.c0, 5 qy.c1
                outputs 0..11 the Fq12 coordinates (ABI order)
                = Bls12::miller_loop([(P, Q.prepare())]) (mod.rs:40-102)
  final_exp     inputs / outputs 0..11 Fq12 coordinates
                = Bls12::final_exponentiation (mod.rs:104-160)

Infinity inputs (miller loop -> one) and f == 0 (final exp -> None) are
lane selects done by the emitted prologue/epilogue, outside the DSL.
"""
from dsl import Prog
from tower import Tower, X_ABS, declare12, get12, set12

ML_MASK = (X_ABS >> 1) & ((1 << 62) - 1)  # bits 61..0 below the leading one of |x| >> 1


def _getR(p):
    return tuple((p.get(n + "0"), p.get(n + "1")) for n in ("rx", "ry", "rz"))


def _setR(p, r):
    for n, v in zip(("rx", "ry", "rz"), r):
        p.set(n + "0", v[0])
        p.set(n + "1", v[1])


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


def ell(T, f, c, px, py):
    """mod.rs:57-69: f.mul_by_014(c2, c1 * P.x, c0 * P.y)"""
    return T.mul_by_014(f, c[2], T.mul_fq(c[1], px), T.mul_fq(c[0], py))


ML_HOMES = {"px": "L", "py": "L", "qx0": "M", "qx1": "M", "qy0": "M", "qy1": "M",
            "rx0": "A", "rx1": "A", "ry0": "A", "ry1": "A", "rz0": "A", "rz1": "A", "f": "A"}


def miller_loop_prog(homes=None):
    homes = dict(ML_HOMES, **(homes or {}))
    p = Prog("miller_loop")
    T = Tower(p)
    pq = ("px", "py", "qx0", "qx1", "qy0", "qy1")
    for i, n in enumerate(pq):
        p.var(n, 1, homes.get(n))
        p.set(n, p.load(i))
    for n in ("rx0", "rx1", "ry0", "ry1", "rz0", "rz1"):
        p.var(n, 1, homes.get(n))
    declare12(p, "f", homes.get("f"))
    one, zero = p.const(1), p.const(0)
    _setR(p, ((p.get("qx0"), p.get("qx1")), (p.get("qy0"), p.get("qy1")), (one, zero)))
    set12(p, "f", ((T.one2(), (zero, zero), (zero, zero)), ((zero, zero),) * 3))

    def line(step):
        f = get12(p, "f")
        r = _getR(p)
        if step == "dbl":
            c, r = doubling_step(T, r)
        else:
            c, r = addition_step(T, r, (p.get("qx0"), p.get("qx1")), (p.get("qy0"), p.get("qy1")))
        f = ell(T, f, c, p.get("px"), p.get("py"))
        set12(p, "f", f)
        _setR(p, r)

    with p.loop(62) as L:
        line("dbl")
        with p.if_bit(ML_MASK, L):
            line("add")
        set12(p, "f", T.sqr12(get12(p, "f")))
    line("dbl")
    f = T.conj12(get12(p, "f"))
    for i, x in enumerate(v for c6 in f for c2 in c6 for v in c2):
        p.store(i, x)
    return p


def exp_by_x(p, T, f, x, tag):
    """exp_by_x (mod.rs:116-121): f^|x| by square-and-multiply (lib.rs:306-324)
    with cyclotomic squarings, then conjugation (x < 0)"""
    base, res = "eb%s_" % tag, "er%s_" % tag
    declare12(p, base, "M")
    declare12(p, res, "A")
    set12(p, base, f)
    set12(p, res, f)
    top = x.bit_length() - 1
    with p.loop(top) as L:
        set12(p, res, T.cyc_sqr(get12(p, res)))
        with p.if_bit(x & ((1 << top) - 1), L):
            set12(p, res, T.mul12(get12(p, res), get12(p, base)))
    return T.conj12(get12(p, res))


def final_exp_prog():
    p = Prog("final_exp")
    T = Tower(p)
    f = (((p.load(0), p.load(1)), (p.load(2), p.load(3)), (p.load(4), p.load(5))),
         ((p.load(6), p.load(7)), (p.load(8), p.load(9)), (p.load(10), p.load(11))))
    # mod.rs:104-160
    f1 = T.conj12(f)
    f2 = T.inv12(f)
    r = T.mul12(f1, f2)
    f2 = r
    r = T.mul12(T.frob12(r, 2), f2)
    x = X_ABS
    y0 = T.cyc_sqr(r)
    y1 = exp_by_x(p, T, y0, x, "a")
    y2 = exp_by_x(p, T, y1, x >> 1, "b")
    y3 = T.conj12(r)
    y1 = T.mul12(y1, y3)
    y1 = T.conj12(y1)
    y1 = T.mul12(y1, y2)
    y2 = exp_by_x(p, T, y1, x, "c")
    y3 = exp_by_x(p, T, y2, x, "d")
    y1 = T.conj12(y1)
    y3 = T.mul12(y3, y1)
    y1 = T.conj12(y1)
    y1 = T.frob12(y1, 3)
    y2 = T.frob12(y2, 2)
    y1 = T.mul12(y1, y2)
    y2 = exp_by_x(p, T, y3, x, "e")
    y2 = T.mul12(y2, y0)
    y2 = T.mul12(y2, r)
    y1 = T.mul12(y1, y2)
    y2 = T.frob12(y3, 1)
    y1 = T.mul12(y1, y2)
    for i, v in enumerate(v for c6 in y1 for c2 in c6 for v in c2):
        p.store(i, v)
    return p
