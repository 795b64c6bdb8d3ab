"""Small generated TEST kernels (not product code): they exercise single
pieces of the emitted code on the GPU against the DSL model
(tests/test_gen_units.py) -- the in-kernel binary GCD, the zero-test select
and Karabina decompression, whose rare branch random pairings never reach.
Both use the final-exponentiation record layout (12 Fq in, 12 Fq out)."""
from dsl import Prog
from tower import TowerLazySq


def dec_prog(lanes=1):
    """load an Fq12, keep its compressed coordinates (a1, a2, b0, b2),
    decompress them (kdec_numden + batch_inv2 over one value + kdec_finish)
    and store the Fq12.  lanes = 2: the lane-pair tower (tower2.Tower2, the
    round-5 lane-pair final exponentiation's decompression)"""
    import kernels
    from tower2 import Tower2
    p = Prog("tdec" if lanes == 1 else "tdec2", lanes, use_norm=True)
    p.binv_ok = True
    T = TowerLazySq(p) if lanes == 1 else Tower2(p)
    V = kernels._Vars(p, lanes)
    (_, a1, a2), (b0, _, b2) = V.load12()
    g = (a1, a2, b0, b2)
    num, den, w = T.kdec_numden(g)
    (iden,) = T.batch_inv2([den], "t")
    V.store12(T.kdec_finish(g, num, iden, w))
    return p


def unit_prog():
    """binv of a product and of a sum, selz with two tests and with one"""
    p = Prog("tunit", use_norm=True)
    xs = [p.load(k) for k in range(12)]
    y = p.mul(xs[0], xs[1])
    i1 = p.binv(y)
    i2 = p.binv(p.red(p.add(xs[2], xs[3])))
    z = p.selz([p.red_full(xs[4]), p.red_full(xs[5])], i1, i2)
    z2 = p.selz([p.red_full(xs[6])], xs[7], xs[8])
    for k, v in enumerate([i1, i2, z, z2, p.mul(i1, y)] + xs[5:12]):
        p.store(k, p.red(v))
    return p
