#!/usr/bin/env python3
"""Simulate one lane of a generated kernel (sim.py) and compare with the DSL
golden model.  python tools/pgen/sim_check.py small|ml|fe"""
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]
import build_gen  # noqa: E402
import dsl  # noqa: E402
import sim  # noqa: E402


def words(xs):
    out = []
    for x in xs:
        out += [(x >> (64 * i)) & (2 ** 64 - 1) for i in range(6)]
    return out


def check(which, seed=5, lane=3, debug=True):
    import kcfg
    f = build_gen.PROGRAMS[which]
    prog, cfg, kname, nmem = f()
    code = f.cache["r"][4]
    if debug:
        code, _ = kcfg.build(prog, type(cfg)(), debug=True)
    trace = []
    rng = random.Random(seed)
    IN, OUT, AUX, WS = 0x100000, 0x200000, 0x300000, 0x400000
    pair = prog.lanes == 2
    lds = {}
    if pair:   # lanes 2*lane, 2*lane+1 handle pairing `lane`
        sim_lane = 2 * lane
    else:
        sim_lane = lane
    if which in ("small", "fe", "fe2", "fez", "fen", "fei"):
        ins = [rng.randrange(dsl.Q) for _ in range(12)]
        rec = [0] * (72 * lane) + words(ins)
        if which == "fei":   # slot 12: Fq 0 of the out record (any value for the check)
            ins.append(rng.randrange(dsl.Q))
        want = dsl.evaluate(prog, {k: ins[k] for k in range(len(ins))}, trace=trace)
        args = [IN, OUT, AUX, lane + 1, WS]
        bufs = {IN: rec}
        if which == "fei":
            bufs[OUT] = [0] * (72 * lane) + words(ins[12:])
    elif which == "mls":
        # P's coordinates and 68 lines of any field values (the loop does not
        # care whether they come from a real G2Prepared)
        import kernels
        ins = [rng.randrange(dsl.Q) for _ in range(2)]
        coeffs = [[rng.randrange(dsl.Q) for _ in range(6)] for _ in range(68)]
        lines = kernels.shared_table_lines(coeffs)
        prec = [0] * (13 * lane) + words(ins) + [0]
        want = dsl.evaluate(prog, {0: ins[0], 1: ins[1], "lines": lines}, trace=trace)
        args = [IN, AUX, OUT, lane + 1, WS]
        table = kernels.shared_table_u64(lines, infinity=False)
        bufs = {IN: prec, AUX: table}
        if getattr(cfg, "lds_table", False):
            # the rows the other 63 lanes of the wave copy into LDS
            t0 = cfg.TABLE_LINES // 8
            for i, w in enumerate(table[t0:]):
                lds[cfg.table_base() + 8 * i] = w & 0xffffffff
                lds[cfg.table_base() + 8 * i + 4] = w >> 32
    elif which == "mlp":
        # lane `lane`'s G2Prepared record (68 lines of six ABI integers, flag 0)
        import kernels
        ins = [rng.randrange(dsl.Q) for _ in range(2)]
        coeffs = [[rng.randrange(dsl.Q) for _ in range(6)] for _ in range(68)]
        prec = [0] * (13 * lane) + words(ins) + [0]
        want = dsl.evaluate(prog, {0: ins[0], 1: ins[1], "lines": kernels.prepared_table_lines(coeffs)},
                            trace=trace)
        rw = cfg.RECORD // 8
        qrec = [0] * (rw * lane) + sum((words(line) for line in coeffs), []) + [0]
        args = [IN, AUX, OUT, lane + 1, WS]
        bufs = {IN: prec, AUX: qrec}
    else:
        # any field values (the loop does not care whether they are on the curve)
        ins = [rng.randrange(dsl.Q) for _ in range(6)]
        prec = [0] * (13 * lane) + words(ins[:2]) + [0]
        qrec = [0] * (25 * lane) + words(ins[2:]) + [0]
        want = dsl.evaluate(prog, {k: ins[k] for k in range(6)}, trace=trace)
        args = [IN, AUX, OUT, lane + 1, WS]
        bufs = {IN: prec, AUX: qrec}
    t = time.time()
    sm = sim.run_lane(code, args, bufs, lane=sim_lane, trace=trace if debug else None, pair=pair, lds=lds)
    got = []
    for k in sorted(want):
        base = OUT + 576 * lane + 48 * k
        got.append(sum(sm.mem.get(base + 4 * j, 0) << (32 * j) for j in range(12)))
    ok = got == [want[k] for k in sorted(want)]
    print("%s lane %d: %s (%d instructions simulated, %.1fs)" % (which, lane, "OK" if ok else "MISMATCH",
                                                              sm.count, time.time() - t))
    if os.environ.get("PGEN_HIST"):
        for m, c in sorted(sm.hist.items(), key=lambda x: -x[1]):
            print("  %-28s %9d" % (m, c))
    return ok


if __name__ == "__main__":
    sys.exit(0 if all(check(w) for w in sys.argv[1:] or ["small"]) else 1)
