"""CPU tests of the kernel generator (tools/pgen), no GPU needed:

  * the DSL programs of the two generated kernels, evaluated with the exact
    limb semantics of the emitted instructions (every lazy bound asserted),
    equal the C oracle's Miller loop / final exponentiation bit for bit --
    for one lane per pairing and for lane pairs;
  * the emitted instruction stream, run by the single-lane / lane-pair
    simulator, reproduces the DSL value of every operation (register
    allocation, spills, control flow, record I/O);
  * the bound system rejects a product whose column sums could overflow.
"""
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PGEN = os.path.join(ROOT, "tools", "pgen")
for p in (PGEN, os.path.join(ROOT, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)

import build_gen  # noqa: E402
import dsl  # noqa: E402
import kernels  # noqa: E402
import sim_check  # noqa: E402
from helpers import random_scalars, rng  # noqa: E402


def _words(a, k):
    return sum(int(w) << (64 * i) for i, w in enumerate(a[6 * k:6 * k + 6]))


@pytest.fixture(scope="module")
def ref_pair(oracle):
    g = rng(11)
    p = oracle.g1_mul_generator(random_scalars(g, 1))
    q = oracle.g2_mul_generator(random_scalars(g, 1))
    ml = oracle.miller_loop_batch(p, oracle.g2_prepare(q))
    fe, _ = oracle.final_exponentiation(ml)
    ins = {k: _words(p[0], k) for k in range(2)}
    ins.update({2 + k: _words(q[0], k) for k in range(4)})
    return ins, [_words(ml[0], k) for k in range(12)], [_words(fe[0], k) for k in range(12)]


@pytest.mark.parametrize("lanes,lazy", [(1, False), (2, False), (1, True)])
def test_dsl_miller_loop_matches_oracle(ref_pair, lanes, lazy):
    ins, ml, _ = ref_pair
    out = dsl.evaluate(kernels.miller_loop_prog(lanes=lanes, lazy=lazy), ins)
    assert [out[k] for k in range(12)] == ml


@pytest.mark.parametrize("lanes,lazy", [(1, False), (2, False), (1, True), (1, "sq")])
def test_dsl_final_exp_matches_oracle(ref_pair, lanes, lazy):
    _, ml, fe = ref_pair
    out = dsl.evaluate(kernels.final_exp_prog(lanes=lanes, lazy=lazy), {k: ml[k] for k in range(12)})
    assert [out[k] for k in range(12)] == fe


def test_dsl_pairing_only_miller_loop_one_lane_gives_the_pairing(ref_pair):
    """the same on one lane per pairing (pa_gen_miller_loop1p)"""
    ins, ml, fe = ref_pair
    f = dsl.evaluate(kernels.miller_loop_prog(pairing_only=True), ins)
    assert [f[k] for k in range(12)] != ml
    out = dsl.evaluate(kernels.final_exp_prog(), {k: f[k] for k in range(12)})
    assert [out[k] for k in range(12)] == fe


def test_wide_values_exact():
    """wide products / normalisation / reduction of the lazy tower equal
    their integer meaning (tower.TowerLazy, dsl.wsop/wnorm/wred)"""
    g = random.Random(9)
    for _ in range(50):
        a, b, c, d = (dsl.gen_fl.limbs(g.randrange(2 * dsl.Q)) for _ in range(4))
        lo, hi = dsl.wide_product([(tuple(a), tuple(b)), (tuple(c), tuple(d))])
        w = dsl.val_of(a) * dsl.val_of(b) + dsl.val_of(c) * dsl.val_of(d)
        assert dsl.val_of(lo) + (dsl.val_of(hi) << (28 * dsl.NL)) == w
        r = dsl.mont_reduce_wide(lo, hi)
        assert (dsl.val_of(r) << (28 * dsl.NL)) % dsl.Q == w % dsl.Q


def test_bounds_reject_column_overflow():
    p = dsl.Prog("t")
    a = p.load(0)
    big = a
    for _ in range(4):
        big = p.add(big, a)   # u = 5
    with pytest.raises(AssertionError):
        p.mul(big, big)       # 25 > 17
    with pytest.raises(AssertionError):
        p.sqr(p.add(p.add(a, a), p.add(a, a)))   # squares need u <= 3


def test_red_brings_any_bound_to_one():
    g = random.Random(3)
    for u in (2, 7, 16):
        for _ in range(200):
            limbs = [0] * dsl.NL
            for _ in range(u):
                x = dsl.gen_fl.limbs(g.randrange(2 * dsl.Q))
                limbs = [a + b for a, b in zip(limbs, x)]
            r = dsl.red_limbs(tuple(limbs))
            assert all(0 <= x <= dsl.MASK for x in r)
            assert dsl.val_of(r) < 2 * dsl.Q
            assert (dsl.val_of(r) - dsl.val_of(limbs)) % dsl.Q == 0


def test_sim_small_program():
    assert sim_check.check("small", debug=True)


# the lazy-reduction variants (mlz / fez) and round 2's split inversion (fei)
# are A/B-only code objects, never loaded by the library: their simulator runs
# (~2.3 min) only with PA_SIM_ALL=1, to keep the CPU suite within minutes
SIM_ALL = os.environ.get("PA_SIM_ALL") == "1"
_ab_only = pytest.mark.skipif(not SIM_ALL, reason="A/B-only code object (PA_SIM_ALL=1 runs it)")


def test_dsl_pairing_only_miller_loop_gives_the_pairing(ref_pair):
    """the pairing-only lane-pair Miller loop (homogeneous G2 steps with their
    own line scaling, kernels.doubling_step_h / addition_step_h): its value
    differs from the reference's Miller value, and the final exponentiation of
    it is the reference's pairing, bit for bit"""
    import tower2
    ins, ml, fe = ref_pair
    prog = tower2.two_pass(lambda: kernels.miller_loop_prog(lanes=2, pairing_only=True), xi_dpp=False)()
    f = dsl.evaluate(prog, ins)
    assert [f[k] for k in range(12)] != ml
    out = dsl.evaluate(kernels.final_exp_prog(), {k: f[k] for k in range(12)})
    assert [out[k] for k in range(12)] == fe


@pytest.mark.parametrize("which", ["ml", "ml2", "ml2p", "ml1p", "ml2ps", pytest.param("mlz", marks=_ab_only)])
def test_sim_miller_loop_kernel(which):
    assert sim_check.check(which, debug=True)


@pytest.mark.slow
@pytest.mark.parametrize("which", ["fe", "fe2", pytest.param("fez", marks=_ab_only)])
def test_sim_final_exp_kernel(which):
    assert sim_check.check(which, debug=True)


def test_generated_code_objects_assemble(tmp_path):
    out = build_gen.build("small", str(tmp_path))
    assert os.path.getsize(out) > 0


def test_coop_schedules_replay_equal_dsl():
    """tools/pgen/coop.py: every cooperative macro's encoded schedule (LIN
    chains, merged products, slot reuse) replayed with the exact limb
    semantics equals the DSL macro it was built from"""
    import coop
    macros, consts = coop.build_all()
    coop.check(macros, consts, trials=1)
    assert sum(len(m.records) for m in macros) < 200


def test_coop_lc_schedules_on_edge_values():
    """the LC (linear-combination) schedules replayed on extreme canonical
    inputs -- arguments 0, 1, q - 1 ... in Montgomery form and the
    non-canonical q and 2q - 1, mixed -- with the kernel's u32 limb arithmetic: no limb leaves
    its F<U> bound, no product column overflows (mont_sop asserts), and the
    field values equal the DSL macro's"""
    import random
    import coop
    import dsl
    from dsl import Loop, If
    assert coop.LC
    macros, consts = coop.build_all()
    rng = random.Random(7)
    # canonical Montgomery forms of edge values, plus non-canonical F<1>
    # inputs a product can hand on: q itself and 2q - 1 (value bound 2q)
    edge = [tuple(dsl.to_mont_limbs(v)) for v in (0, 1, dsl.Q - 1, dsl.Q - 2, (dsl.Q - 1) // 2)]
    edge += [tuple(dsl.gen_fl.limbs(dsl.Q)), tuple(dsl.gen_fl.limbs(2 * dsl.Q - 1))]
    for m in macros:
        refs = set()

        def collect(block):
            for it in block.items:
                if isinstance(it, (Loop, If)):
                    collect(it.body)
                elif it.kind == "arg":
                    refs.add(it.imm)
        collect(m.prog.root)
        for trial in range(3):
            args = {r: edge[(trial + k) % len(edge)] if trial < 2 else rng.choice(edge)
                    for k, r in enumerate(sorted(refs))}
            want = dsl.evaluate(m.prog, args)
            got = coop.replay(m, consts, args)
            for k in want:
                assert dsl.val_of(got[k]) % dsl.Q == dsl.val_of(want[k]) % dsl.Q, (m.name, k)
                assert max(got[k]) < (1 << 28) and dsl.val_of(got[k]) < 2 * dsl.Q, (m.name, k)


# ---- round 2: value bounds, carry normalization, add fusion, subtraction tables ----
def test_subtraction_tables_dominate_subtrahends():
    """SUBC[(u, v)]: a multiple of q whose limbs 0..12 are >= u (2^28 - 1) and whose
    top limb covers any value below v 2q (top limb < v 2^18); its value bound is
    strict (tools/gen_fl.py sub_constant2)"""
    import gen_fl
    for u in (1, 2, 3, 5):
        for v in (1, 2, 6, 12):
            c, ul, uv = gen_fl.sub_constant2(u, v)
            val = dsl._val_of(c)
            assert val % dsl.Q == 0
            assert all(x >= u * dsl.MASK for x in c[:13]) and c[13] >= v << 18
            assert val < uv * 2 * dsl.Q and all(x <= ul * dsl.MASK for x in c)
            # the largest subtrahend of those bounds stays non-negative limb-wise
            top = (v * 2 * dsl.Q - 1) >> (28 * 13)
            assert c[13] >= min(top, u * dsl.MASK)


def test_norm_keeps_value_and_limits_limbs():
    r = random.Random(3)
    for _ in range(200):
        x = tuple(r.randrange(15 * dsl.MASK) for _ in range(13)) + (r.randrange(1 << 22),)
        y = dsl.norm_limbs(x)
        assert dsl._val_of(y) == dsl._val_of(x)
        assert all(v <= dsl.MASK for v in y[:13])


def test_products_reject_large_value_bounds():
    p = dsl.Prog("t", use_norm=True)
    a = p._op("const", [], 1, imm=tuple([0] * 14), vb=30)
    with pytest.raises(AssertionError, match="value bound"):
        p.mul(a, a)
    b = p._op("const", [], 1, imm=tuple([0] * 14), vb=20)
    p.mul(b, b)          # 400 <= VB_PROD


def test_red_becomes_norm_only_for_small_value_bounds():
    p = dsl.Prog("t", use_norm=True)
    x = p._op("const", [], 1, imm=tuple([0] * 14))
    s = p.add(p.add(x, x), x)                 # u = vb = 3
    assert p.red(s).u == 1 and p.cur.items[-1].kind == "norm"
    big = x
    for _ in range(dsl.VN):
        big = p.add(big, x)                   # vb = VN + 1
    r = p.red(big)
    assert p.cur.items[-1].kind == "red" and r.vb == 1
    q = dsl.Prog("t")                         # coop / lane-pair programs: always the full reduction
    y = q._op("const", [], 1, imm=tuple([0] * 14))
    q.red(q.add(y, y))
    assert q.cur.items[-1].kind == "red"


def test_fuse_adds_preserves_values():
    r = random.Random(5)
    p = dsl.Prog("t", use_norm=True)
    a, b, c, d = (p.load(k) for k in range(4))
    t = p.add(a, b)
    u = p.add(t, c)                            # add3
    w = p.add(d, d)
    w = p.add(w, w)                            # shl 2
    z = p.add(w, u)                            # shladd
    v = p.add(p.add(c, c), a)                  # shladd 1
    for k, val in enumerate((u, z, v)):
        p.store(k, p.red(val))
    ins = {k: r.randrange(dsl.Q) for k in range(4)}
    want = dsl.evaluate(p, ins)
    n = dsl.fuse_adds(p)
    kinds = [it.kind for it in p.root.items]
    assert n >= 3 and "add3" in kinds and "shladd" in kinds
    assert dsl.evaluate(p, ins) == want
    Q = dsl.Q
    assert want[0] == (ins[0] + ins[1] + ins[2]) % Q
    assert want[1] == (4 * ins[3] + ins[0] + ins[1] + ins[2]) % Q


# ---- round 2: the final exponentiation split around a binary-GCD inversion ----
def test_dsl_split_final_exp_composes(ref_pair):
    """norm program -> Fq inverse (R = 2^384 Montgomery records) -> inv program
    equals the one-kernel final exponentiation and the oracle (mod.rs:104-160)"""
    _, ml, fe = ref_pair
    ins = {k: ml[k] for k in range(12)}
    nrm = dsl.evaluate(kernels.final_exp_prog(lazy="sq", split="norm"), dict(ins))
    assert sorted(nrm) == [0] and nrm[0] != 0
    r = 1 << 384
    ins[12] = r * r * pow(nrm[0], -1, dsl.Q) % dsl.Q
    out = dsl.evaluate(kernels.final_exp_prog(lazy="sq", split="inv"), ins)
    assert [out[k] for k in range(12)] == fe


def test_split_final_exp_saves_the_fermat_chain(monkeypatch):
    """round 2's split form against round 2's one-kernel form (Fermat
    inversion, Granger-Scott exp_by_x: PGEN_KARABINA=0), and round 3's
    one-kernel form (in-kernel binary GCD, compressed squarings) below both"""
    import random
    g = random.Random(2)
    ins = {k: g.randrange(dsl.Q) for k in range(13)}
    macs = {}
    for split in (None, "norm", "inv"):
        st = dsl.Stats()
        monkeypatch.setenv("PGEN_KARABINA", "0")
        dsl.evaluate(kernels.final_exp_prog(lazy="sq", split=split), dict(ins), st)
        macs[split] = build_gen.macs(st.counts)
    monkeypatch.setenv("PGEN_KARABINA", "1")
    st = dsl.Stats()
    dsl.evaluate(kernels.final_exp_prog(lazy="sq"), dict(ins), st)
    kara = build_gen.macs(st.counts)
    # the 463-product Fermat chain (~181 k limb MACs) leaves; the norm kernel is ~1 % of the FE
    assert macs[None] - macs["inv"] > 170000
    assert macs["norm"] < 0.01 * macs[None]
    # compressed squarings: ~17 % fewer limb MACs than the split form
    assert kara < 0.85 * macs["inv"]


def test_sim_fe_norm_kernel():
    assert sim_check.check("fen", debug=True)


@pytest.mark.slow
@_ab_only
def test_sim_fe_inv_kernel():
    assert sim_check.check("fei", debug=True)


# ---- round 3: compressed squaring, in-kernel binary GCD, zero-test select ----
def _cyclotomic(seed):
    """a random element of the cyclotomic subgroup (the easy part of the final
    exponentiation applied to a random Fq12), Python model"""
    import pymodel as pm
    g = random.Random(seed)
    f = tuple(tuple((g.randrange(dsl.Q), g.randrange(dsl.Q)) for _ in range(3)) for _ in range(2))
    t = pm.f12mul(pm.f12conj(f), pm.f12inv(f))
    return pm.f12mul(pm.f12pow(t, dsl.Q * dsl.Q), t)


def _b0_zero_element():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "karabina_b0zero.json")) as fh:
        f = json.load(fh)["f"]
    return tuple(tuple((x[0], x[1]) for x in c) for c in f)


def _model_ksqr(g):
    import pymodel as pm

    def sc(k, a):
        return ((k * a[0]) % dsl.Q, (k * a[1]) % dsl.Q)
    a1, a2, b0, b2 = g
    sq = lambda x: pm.f2mul(x, x)  # noqa: E731
    return (pm.f2sub(sc(3, pm.f2add(sq(b0), pm.f2xi(sq(a2)))), sc(2, a1)),
            pm.f2sub(sc(3, pm.f2add(sq(a1), pm.f2xi(sq(b2)))), sc(2, a2)),
            pm.f2add(sc(6, pm.f2xi(pm.f2mul(a1, b2))), sc(2, b0)),
            pm.f2add(sc(6, pm.f2mul(b0, a2)), sc(2, b2)))


def test_karabina_formulas_on_the_model():
    """tower.Tower.ksqr's formulas square the compressed coordinates of
    cyclotomic elements (against full squaring in the Python model), and the
    element with b0 = 0 (tests/golden/karabina_b0zero.json) is really in the
    cyclotomic subgroup and satisfies the b0 = 0 decompression identity
    b1 a2 = 2 a1 b2 that kdec_numden's select relies on"""
    import pymodel as pm
    for f in (_cyclotomic(1), _cyclotomic(2), _b0_zero_element()):
        assert pm.f12mul(f, pm.f12conj(f)) == pm.F12ONE
        g = (f[0][1], f[0][2], f[1][0], f[1][2])
        for _ in range(3):
            f = pm.f12mul(f, f)
            g = _model_ksqr(g)
            assert g == (f[0][1], f[0][2], f[1][0], f[1][2])
    z = _b0_zero_element()
    (a0, a1, a2), (b0, b1, b2) = z
    assert b0 == (0, 0) and a2 != (0, 0)
    assert pm.f2mul(b1, a2) == pm.f2add(pm.f2mul(a1, b2), pm.f2mul(a1, b2))


def _dec_prog():
    import unit_progs
    return unit_progs.dec_prog()


def _abi_words(f):
    """plain Fq12 -> the 12 canonical Montgomery (R = 2^384) integers, ABI order"""
    R384 = (1 << 384) % dsl.Q
    return [(x * R384) % dsl.Q for c6 in f for c2 in c6 for x in c2]


@pytest.mark.parametrize("lanes", [1, 2])
@pytest.mark.parametrize("which", ["random", "b0_zero", "identity"])
def test_dsl_karabina_decompression(which, lanes):
    """the DSL decompression (both branches of the b0 == 0 select, and the
    identity whose inversion input is 0) rebuilds the element exactly, on
    one lane and on the lane-pair tower"""
    import pymodel as pm
    import unit_progs
    f = {"random": lambda: _cyclotomic(3), "b0_zero": _b0_zero_element, "identity": lambda: pm.F12ONE}[which]()
    ins = _abi_words(f)
    out = dsl.evaluate(unit_progs.dec_prog(lanes=lanes), {k: ins[k] for k in range(12)})
    assert [out[k] for k in range(12)] == ins


def test_binv_model_is_the_inverse():
    """dsl.binv_limbs (the emitted binary GCD's exact limbs) is a^-1 R' for
    aR' = x, 0 for x = 0 mod q, over random lazy inputs and edge values"""
    g = random.Random(4)
    R = dsl.R
    vals = [0, dsl.Q, 1, dsl.Q - 1, dsl.Q + 1, 2 * dsl.Q - 1, R % dsl.Q, (1 << 380)] + \
        [g.randrange(2 * dsl.Q) for _ in range(200)]
    for v in vals:
        out = dsl.val_of(dsl.binv_limbs(tuple(dsl.gen_fl.limbs(v))))
        assert out < 2 * dsl.Q
        a = v * pow(R, -1, dsl.Q) % dsl.Q
        assert out % dsl.Q == (pow(a, -1, dsl.Q) * R % dsl.Q if a else 0)


def _unit_prog():
    import unit_progs
    return unit_progs.unit_prog()


def _sim_run(prog, ins, lane=3):
    import kcfg
    import sim
    cfg = kcfg.FinalExpCfg()
    cfg.name = prog.name
    code, _ = kcfg.build(prog, cfg, debug=True)
    trace = []
    want = dsl.evaluate(prog, {k: ins[k] for k in range(12)}, trace=trace)
    IN, OUT, AUX, WS = 0x100000, 0x200000, 0x300000, 0x400000
    sm = sim.run_lane(code, [IN, OUT, AUX, lane + 1, WS], {IN: [0] * (72 * lane) + sim_check.words(ins)},
                      lane=lane, trace=trace)
    got = [sum(sm.mem.get(OUT + 576 * lane + 48 * k + 4 * j, 0) << (32 * j) for j in range(12)) for k in range(12)]
    return got, [want[k] for k in range(12)]


@pytest.mark.parametrize("case", range(4))
def test_sim_binv_and_selz(case):
    """the emitted binary GCD and zero-test select, run by the simulator (with
    its gfx950 VALU-SGPR wait-state check), equal the DSL model limb for limb:
    random inputs, zero tests true for (0, 0), inverses of 0 and of q"""
    g = random.Random(7 + case)
    ins = [g.randrange(dsl.Q) for _ in range(12)]
    if case == 1:
        ins[4] = ins[5] = ins[6] = 0
    if case == 2:
        ins[0] = 0
        ins[4] = 0
    if case == 3:
        ins[2] = dsl.Q - ins[3]
        ins[6] = 0
    got, want = _sim_run(_unit_prog(), ins)
    assert got == want
    assert got[4] == ((1 << 384) % dsl.Q if ins[0] and ins[1] else 0)


def test_sim_karabina_decompression_b0_zero():
    """the emitted decompression on the b0 = 0 element (the select's rare
    branch) equals the DSL model and the element itself"""
    ins = _abi_words(_b0_zero_element())
    got, want = _sim_run(_dec_prog(), ins)
    assert got == want == ins


def test_sim_karabina_decompression_b0_zero_lane_pairs():
    """the same for the lane-pair program, both lanes simulated in lockstep"""
    import kcfg
    import sim
    import unit_progs
    prog = unit_progs.dec_prog(lanes=2)
    cfg = kcfg.FinalExpCfg2()
    cfg.name = prog.name
    code, _ = kcfg.build(prog, cfg, debug=True)
    ins = _abi_words(_b0_zero_element())
    trace = []
    want = dsl.evaluate(prog, {k: ins[k] for k in range(12)}, trace=trace)
    lane = 3
    IN, OUT, AUX, WS = 0x100000, 0x200000, 0x300000, 0x400000
    sm = sim.run_lane(code, [IN, OUT, AUX, lane + 1, WS], {IN: [0] * (72 * lane) + sim_check.words(ins)},
                      lane=2 * lane, trace=trace, pair=True)
    got = [sum(sm.mem.get(OUT + 576 * lane + 48 * k + 4 * j, 0) << (32 * j) for j in range(12)) for k in range(12)]
    assert got == [want[k] for k in range(12)] == ins


def test_local_homes_free_dead_variables():
    """emit.Emitter.index_vars: a variable written first inside a loop body and
    used only there gets its home only in that body (round 3's looped hard
    part relies on it to reuse AGPR homes between its phases)"""
    import emit
    import kcfg
    p = dsl.Prog("t", use_norm=True)
    x = p.load(0)
    p.var("outer", 1, "A")
    p.set("outer", x)
    with p.loop(3):
        p.var("inner", 1, "A")
        p.set("inner", p.mul(p.get("outer"), p.get("outer")))
        p.set("outer", p.get("inner"))
    p.store(0, p.get("outer"))
    em = emit.Emitter(p, kcfg.FinalExpCfg())
    em.run_block(p.root, top=True)
    loop_body = [it for it in p.root.items if isinstance(it, dsl.Loop)][0].body
    assert em.local_vars.get(id(loop_body)) == {"inner"}
