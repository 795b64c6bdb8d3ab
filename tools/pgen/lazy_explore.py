#!/usr/bin/env python3
"""Explore which TowerLazy overrides pay off: build the ML / FE programs with
a subset of the lazy overrides, emit them, simulate one lane and print the
dynamic instruction mix (the lone-wave kernels are issue-bound: ~one
instruction per quad-cycle, plus memory waits).

  python tools/pgen/lazy_explore.py ml|fe  mul2,mul6,mul_by_01,fq4_sqr ...
"""
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]
import dsl  # noqa: E402
import kcfg  # noqa: E402
import kernels  # noqa: E402
import sim  # noqa: E402
import tower  # noqa: E402


def lazy_tower(flags):
    over = {k: getattr(tower.TowerLazy, k) for k in flags}
    return type("TowerSel", (tower.TowerLazy,), {k: getattr(tower.Tower, k) for k in
                                                ("mul2", "mul6", "mul_by_01", "fq4_sqr") if k not in over})


def run(which, flags):
    T = lazy_tower(flags)
    orig = kernels.TowerLazy
    kernels.TowerLazy = T
    try:
        prog = kernels.miller_loop_prog(lazy=True) if which == "ml" else kernels.final_exp_prog(lazy=True)
    finally:
        kernels.TowerLazy = orig
    dsl.check_scopes(prog)
    cfg = kcfg.MillerLoopCfg() if which == "ml" else kcfg.FinalExpCfg()
    cfg.name = "x"
    code, em = kcfg.build(prog, cfg)
    rng = random.Random(5)
    lane = 3
    IN, OUT, AUX, WS = 0x100000, 0x200000, 0x300000, 0x400000

    def words(xs):
        return [(x >> (64 * i)) & (2 ** 64 - 1) for x in xs for i in range(6)]
    if which == "fe":
        ins = [rng.randrange(dsl.Q) for _ in range(12)]
        bufs = {IN: [0] * (72 * lane) + words(ins)}
        args = [IN, OUT, AUX, lane + 1, WS]
    else:
        ins = [rng.randrange(dsl.Q) for _ in range(6)]
        bufs = {IN: [0] * (13 * lane) + words(ins[:2]) + [0], AUX: [0] * (25 * lane) + words(ins[2:]) + [0]}
        args = [IN, AUX, OUT, lane + 1, WS]
    want = dsl.evaluate(prog, {k: ins[k] for k in range(len(ins))})
    t = time.time()
    sm = sim.run_lane(code, args, bufs, lane=lane)
    got = [sum(sm.mem.get(OUT + 576 * lane + 48 * k + 4 * j, 0) << (32 * j) for j in range(12)) for k in range(12)]
    h = sm.hist
    tot = sum(v for k, v in h.items() if k not in ("mark", "label"))
    mad = h.get("v_mad_u64_u32", 0)
    gl = sum(v for k, v in h.items() if k.startswith("global_load"))
    ds = sum(v for k, v in h.items() if k.startswith("ds_"))
    print("%s %-28s %s instr %8d mad %8d other %8d ds %6d gload %6d (%.0fs)" % (
        which, ",".join(flags) or "-", "OK " if got == [want[k] for k in range(12)] else "BAD", tot, mad,
        tot - mad, ds, gl, time.time() - t))


if __name__ == "__main__":
    which = sys.argv[1]
    for spec in sys.argv[2:]:
        run(which, [f for f in spec.split(",") if f and f != "-"])
