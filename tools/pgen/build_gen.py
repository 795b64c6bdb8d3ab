#!/usr/bin/env python3
"""Build the generated pairing kernels: DSL programs -> register allocation
+ emission -> gfx950 assembly -> code object (pairing_amd/lib/*.hsaco).

  python tools/pgen/build_gen.py [small|ml|fe ...] [--outdir DIR]
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, os.path.dirname(HERE)]

import dsl  # noqa: E402
import kcfg  # noqa: E402
import kernels  # noqa: E402
import render  # noqa: E402
from tower import Tower, declare12, get12, set12  # noqa: E402


def small_prog():
    p = dsl.Prog("small")
    T = Tower(p)
    f = (((p.load(0), p.load(1)), (p.load(2), p.load(3)), (p.load(4), p.load(5))),
         ((p.load(6), p.load(7)), (p.load(8), p.load(9)), (p.load(10), p.load(11))))
    declare12(p, "acc")
    set12(p, "acc", f)
    with p.loop(3) as L:
        set12(p, "acc", T.cyc_sqr(get12(p, "acc")))
        with p.if_bit(0b101, L):
            set12(p, "acc", T.mul12(get12(p, "acc"), get12(p, "acc")))
    y = T.mul12(get12(p, "acc"), f)
    for i, v in enumerate(v for c6 in y for c2 in c6 for v in c2):
        p.store(i, v)
    return p


def cyc_probe_prog(iters=None):
    """timing probe (not a product kernel): iters cyclotomic squarings in a loop,
    the final exponentiation's hot loop body alone (tools/pgen/gpu_check.py cyc)"""
    from tower import TowerLazySq
    iters = iters or int(os.environ.get("PGEN_CYC_ITERS", "100"))
    p = dsl.Prog("cyc")
    T = TowerLazySq(p)
    f = (((p.load(0), p.load(1)), (p.load(2), p.load(3)), (p.load(4), p.load(5))),
         ((p.load(6), p.load(7)), (p.load(8), p.load(9)), (p.load(10), p.load(11))))
    declare12(p, "acc", "A")
    set12(p, "acc", f)
    body = os.environ.get("PGEN_CYC_BODY", "cyc")
    with p.loop(iters):
        if body == "cyc":
            set12(p, "acc", T.cyc_sqr(get12(p, "acc")))
        else:   # k Fq4 squarings (a third of a cyclotomic square each): code-size probe
            (a0, a1, a2), (b0, b1, b2) = get12(p, "acc")
            pairs = [(a0, b1), (b0, a2), (a1, b2)]
            outs = [T.fq4_sqr(x, y) for x, y in pairs[:int(body[3:])]] + pairs[int(body[3:]):]
            (a0, b1), (b0, a2), (a1, b2) = outs
            set12(p, "acc", ((a0, a1, a2), (b0, b1, b2)))
    for i, v in enumerate(v for c6 in get12(p, "acc") for c2 in c6 for v in c2):
        p.store(i, v)
    return p


def _with(mod, name, value, progf):
    """progf() with mod.name = value while it builds"""
    def f():
        old = getattr(mod, name)
        setattr(mod, name, value)
        try:
            return progf()
        finally:
            setattr(mod, name, old)
    return f


def _mk(progf, cfgc, kname):
    cache = {}

    def f():
        if "r" not in cache:
            prog = progf()
            dsl.check_scopes(prog)
            cfg = cfgc()
            cfg.name = kname
            code, em = kcfg.build(prog, cfg)
            cache["r"] = (prog, cfg, kname, max(len(em.mslot), 1), code, em)
        prog, cfg, kn, nmem, _, _ = cache["r"]
        return prog, cfg, kn, nmem
    f.cache = cache
    return f


PROGRAMS = {
    "small": _mk(small_prog, kcfg.FinalExpCfg, "pa_gen_small"),
    "cyc": _mk(cyc_probe_prog, kcfg.FinalExpCfg, "pa_gen_cyc"),
    "ml": _mk(kernels.miller_loop_prog, kcfg.MillerLoopCfg, "pa_gen_miller_loop"),
    # default final exponentiation: lazy Fq4 squarings only (tower.TowerLazySq, -1.5 % time);
    # PGEN_FE_LAZY=0 / 1 builds the plain / fully lazy tower instead (A/B experiments)
    "fe": _mk(lambda: kernels.final_exp_prog(lazy={"sq": "sq", "0": False, "1": True}[os.environ.get("PGEN_FE_LAZY", "sq")]),
              kcfg.FinalExpCfg, "pa_gen_final_exp"),
    # round 2's final exponentiation split around a separate base-field
    # inversion (no longer loaded by gen_launch.hip; built only on request)
    "fen": _mk(lambda: kernels.final_exp_prog(lazy="sq", split="norm"), kcfg.FinalExpCfg, "pa_gen_fe_norm"),
    "fei": _mk(lambda: kernels.final_exp_prog(lazy="sq", split="inv"), kcfg.FinalExpCfg, "pa_gen_fe_inv"),
    "ml2": _mk(__import__("tower2").two_pass(lambda: kernels.miller_loop_prog(lanes=2), xi_dpp=False),
                kcfg.MillerLoopCfg2,
                "pa_gen_miller_loop2"),
    # e(P, Q) only (pa_pairing_batch / multi_pairing): homogeneous G2 steps with their own line scaling
    "ml2p": _mk(__import__("tower2").two_pass(lambda: kernels.miller_loop_prog(lanes=2, pairing_only=True),
                                               xi_dpp=False),
                kcfg.MillerLoopCfg2p, "pa_gen_miller_loop2p"),
    # A/B only: ml2p with the signed-operand Fq2 squaring (tower2.SQR_SIGNED)
    "ml2ps": _mk(_with(__import__("tower2"), "SQR_SIGNED", True, __import__("tower2").two_pass(
        lambda: kernels.miller_loop_prog(lanes=2, pairing_only=True), xi_dpp=False)),
        kcfg.MillerLoopCfg2p, "pa_gen_miller_loop2p"),
    # the same on one lane per pairing (the default in (PA_PAIR_MAX, PA_ONE_MAX], variant 3)
    "ml1p": _mk(lambda: kernels.miller_loop_prog(pairing_only=True), kcfg.MillerLoopCfg1p, "pa_gen_miller_loop1p"),
    # one G2Prepared shared by the whole batch: the line table in place of G2 arithmetic
    "mls": _mk(kernels.miller_loop_shared_prog, kcfg.MillerLoopSharedCfg, "pa_gen_miller_loop_shared"),
    # a G2Prepared per pairing (the north-star call): the lines read from each lane's record
    "mlp": _mk(kernels.miller_loop_prepared_prog, kcfg.MillerLoopPreparedCfg, "pa_gen_miller_loop_prepared"),
    # test-only kernels (tools/pgen/unit_progs.py, tests/test_gen_units.py)
    "tdec": _mk(lambda: __import__("unit_progs").dec_prog(), kcfg.FinalExpCfg, "pa_gen_tdec"),
    "tunit": _mk(lambda: __import__("unit_progs").unit_prog(), kcfg.FinalExpCfg, "pa_gen_tunit"),
    "tdec2": _mk(lambda: __import__("unit_progs").dec_prog(lanes=2), kcfg.FinalExpCfg2, "pa_gen_tdec2"),
    "fe2": _mk(__import__("tower2").two_pass(lambda: kernels.final_exp_prog(lanes=2)), kcfg.FinalExpCfg2,
                "pa_gen_final_exp2"),
    # lazy reduction (tower.TowerLazy): wide products, one reduction per output Fq
    # (measured slower; built only on request for A/B runs)
    "mlz": _mk(lambda: kernels.miller_loop_prog(lazy=True), kcfg.MillerLoopCfg, "pa_gen_miller_loop_lazy"),
    "fez": _mk(lambda: kernels.final_exp_prog(lazy=True), kcfg.FinalExpCfg, "pa_gen_final_exp_lazy"),
}
FILES = {"small": "pa_gen_small.hsaco", "cyc": "pa_gen_cyc.hsaco", "ml": "pa_gen_miller_loop.hsaco", "fe": "pa_gen_final_exp.hsaco",
         "mls": "pa_gen_miller_loop_shared.hsaco", "mlp": "pa_gen_miller_loop_prepared.hsaco",
         "fen": "pa_gen_fe_norm.hsaco", "fei": "pa_gen_fe_inv.hsaco",
         "ml2": "pa_gen_miller_loop2.hsaco", "ml2p": "pa_gen_miller_loop2p.hsaco", "ml1p": "pa_gen_miller_loop1p.hsaco", "ml2ps": "pa_gen_miller_loop2p.hsaco", "fe2": "pa_gen_final_exp2.hsaco",
         "mlz": "pa_gen_miller_loop_lazy.hsaco", "fez": "pa_gen_final_exp_lazy.hsaco",
         "tdec": "test/pa_gen_tdec.hsaco", "tunit": "test/pa_gen_tunit.hsaco", "tdec2": "test/pa_gen_tdec2.hsaco"}


def build(which, outdir):
    t = time.time()
    f = PROGRAMS[which]
    f()
    prog, cfg, kname, nmem, code, em = f.cache["r"]
    import emit
    asm = render.kernel_asm(kname, code, em.lds_bytes, lanes=prog.lanes,
                            nvgpr=256 if prog.lanes == 1 else min(256, -(-(emit.VSLOT0 + 14 * em.NV) // 4) * 4),
                            mem_slots=nmem, nsgpr=getattr(cfg, "nsgpr", 96))
    out = os.path.join(outdir, FILES[which])
    os.makedirs(os.path.dirname(out), exist_ok=True)
    render.assemble(asm, out, os.path.join(ROOT, "build", "pgen"))
    nv = sum(1 for t in code if t[0].startswith("v_"))
    print("%s: %d instructions (%d VALU), %d M slots, %.1fs  %s" % (
        out, len(code), nv, nmem, time.time() - t,
        {k[4:]: int(v) for k, v in sorted(em.stats.items()) if k.startswith("dyn_reload") or k.startswith("dyn_spill")}))
    return out


def macs(counts):
    """28x28-bit limb multiply-accumulates (v_mad_u64_u32 / v_mad_i64_i32) of
    one pairing, from the DSL's dynamic op counts: a K-term product leaf is
    196 (K + 1) (K products + one Montgomery reduction), a square 392 (it is
    emitted as a one-term product), red() 30; lazy reduction: a K-term wide
    product 196 K, its reduction wred() 222 (196 + 26 column additions)."""
    n = 0
    for k, v in counts.items():
        if k.startswith("sop") and k[3:].isdigit():
            n += 196 * (int(k[3:]) + 1) * v
        elif k.startswith("wsop") and k[4:].isdigit():
            n += 196 * int(k[4:]) * v
    return n + 392 * counts.get("sqr", 0) + 30 * counts.get("red", 0) + 222 * counts.get("wred", 0)


def write_work_json(outdir):
    """per-kernel algorithmic work of one pairing (bench.py's roofline)"""
    import json
    import random
    rng = random.Random(1)
    out = {}
    for key, name, nin in (("ml", "miller_loop", 6), ("fe", "final_exp", 12), ("fen", "fe_norm", 12),
                           ("fei", "fe_inv", 13), ("mls", "miller_loop_shared", 2),
                           ("mlp", "miller_loop_prepared", 2),
                           ("ml2", "miller_loop_lane_pairs", 6), ("fe2", "final_exp_lane_pairs", 12),
                           ("ml2p", "miller_loop_lane_pairs_pairing_only", 6),
                           ("ml1p", "miller_loop_pairing_only", 6)):
        if key in ("fen", "fei", "mls", "mlp", "ml2", "fe2", "ml2p", "ml1p") and not PROGRAMS[key].cache:
            continue
        prog = PROGRAMS[key]()[0]
        st = dsl.Stats()
        ins = {k: rng.randrange(dsl.Q) for k in range(nin)}
        if key in ("mls", "mlp"):
            coeffs = [[rng.randrange(dsl.Q) for _ in range(6)] for _ in range(68)]
            ins["lines"] = (kernels.shared_table_lines if key == "mls" else kernels.prepared_table_lines)(coeffs)
        dsl.evaluate(prog, ins, st)
        em = PROGRAMS[key].cache["r"][5]
        # instructions one lane executes (exact: the loop trip counts and branch
        # masks are static, the emitter weights every instruction by them)
        # lane pairs: the DSL counts and the emitter's estimate are per lane;
        # a pairing is two lanes' work
        lanes = prog.lanes
        out[name] = {"limb_macs": lanes * macs(st.counts), "ops": st.counts,
                     "instructions": round(lanes * em.dyn_instr), "lanes_per_pairing": lanes}
    with open(os.path.join(outdir, "pa_gen_work.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def main():
    args = sys.argv[1:]
    outdir = os.path.join(ROOT, "pairing_amd", "lib")
    if "--outdir" in args:
        i = args.index("--outdir")
        outdir = args[i + 1]
        del args[i:i + 2]
    os.makedirs(outdir, exist_ok=True)
    meta = {}
    for w in args or ["ml", "fe", "ml2", "fe2", "mls", "mlp", "ml2p", "ml1p"]:
        build(w, outdir)
        meta[w] = PROGRAMS[w].cache["r"][3]
    if "ml" in meta and "fe" in meta or "ml2" in meta and "fe2" in meta:
        for k in ("ml", "fe", "ml2", "fe2", "mls", "mlp", "ml2p", "ml1p"):
            PROGRAMS[k]()   # every program the work file describes
        write_work_json(outdir)
    if all(k in meta for k in ("ml", "fe", "ml2", "fe2", "mls", "mlp", "ml2p", "ml1p")):
        hdr = os.path.join(ROOT, "pairing_amd", "csrc", "pa_gen_meta.h")
        with open(hdr, "w") as f:
            f.write("// GENERATED by tools/pgen/build_gen.py -- spill workspace per wave (M slots)\n#pragma once\n")
            for k, name in (("ml", "MILLER_LOOP"), ("fe", "FINAL_EXP"), ("ml2", "MILLER_LOOP2"), ("fe2", "FINAL_EXP2"),
                            ("mls", "MILLER_LOOP_SHARED"), ("mlp", "MILLER_LOOP_PREPARED"),
                            ("ml2p", "MILLER_LOOP2P"), ("ml1p", "MILLER_LOOP1P")):
                f.write("#define PA_GEN_%s_MEM_SLOTS %d\n" % (name, meta[k]))


if __name__ == "__main__":
    main()
