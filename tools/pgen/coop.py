#!/usr/bin/env python3
"""Cooperative (one wave per pairing) macro-operations for small batches.

The one-lane generated kernels run a pairing's ~3.9 M + 5.4 M instructions
on one lane: ~20 ms whatever the batch size up to 2^16 -- the wrong shape for
a verifier checking a handful of pairs (mod.rs:49-95).  Here the tower and
line operations of the SAME DSL code (kernels.py doubling_step /
addition_step / ell, tower.py sqr12 / mul12 / cyc_sqr / frob12 / inv12) are
each flattened into a dataflow graph and scheduled over the 64 lanes of one
wave: every step runs up to 64 independent field operations of one kind,
one per lane, on operands held in LDS.  A macro's latency is its critical
path (one product level for a cyclotomic squaring: nine Fq2 squarings side
by side) instead of its operation count.  kernels_coop.hip strings the
macros together in the reference's order (mod.rs:40-160) with plain HIP
control flow.

Step kinds (one leaf per step, so a wave never diverges inside a product):
  P1  a*b            (fl_mul_leaf)          P2  a*b + c*d  (fl_sop2_leaf)
  SQ  a^2            (fl_sqr_leaf)          LIN add / sub / neg / red
  INV a^-1           (one lane: bgcd.h binary GCD on the 12-word core)
The base-field inversion (fq.rs:849-902) is one INV op instead of
Tower.inv_fq's Fermat chain (same field value, canonical).

Operands are LDS slots named (group, index): group 0 = absolute (constants,
then the macro's temporaries), groups 1-5 = the operand areas A-E the caller
passes (uniform base slots).  Lane record (u16 x 6):
  op | imm << 4, dst, src0, src1, src2, src3      with slot = group << 12 | index

Output: pairing_amd/csrc/coop_prog.h.  `--check` replays every macro's
schedule with the exact limb semantics of dsl.evaluate and compares it with
the DSL macro itself.

  python tools/pgen/coop.py [--check]
"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, os.path.dirname(HERE)]

import dsl  # noqa: E402
import kernels  # noqa: E402
from dsl import Loop, If, Prog  # noqa: E402
from tower import Tower, X_ABS  # noqa: E402

LANES = 64
K_LIN, K_P1, K_P2, K_SQ, K_INV = range(5)
KIND_NAME = ["LIN", "P1", "P2", "SQ", "INV"]
L_ADD, L_SUB, L_NEG, L_RED = range(4)
# latency estimates (instructions) for the list scheduler's priorities
COST = {K_LIN: 60, K_P1: 540, K_P2: 740, K_SQ: 460, K_INV: 9000, "arg": 0, "ret": 0}
GA, GB, GC, GD, GE = 1, 2, 3, 4, 5   # operand areas


class VmTower(Tower):
    """Tower with the base-field inversion as one op (dsl.Prog.inv)"""

    def inv_fq(self, a, tag):
        return self.p.inv(a)


# ---------------- macro definitions (DSL) ----------------
def _args(p, g, n):
    return [p.arg(g, i) for i in range(n)]


def _fq2s(xs):
    return [(xs[2 * i], xs[2 * i + 1]) for i in range(len(xs) // 2)]


def _f12(xs):
    x = _fq2s(xs)
    return ((x[0], x[1], x[2]), (x[3], x[4], x[5]))


def _flat12(f):
    return [v for c6 in f for c2 in c6 for v in c2]


def _rets(p, g, vals):
    for i, v in enumerate(vals):
        p.ret(g, i, p.red(v))


def m_dbl():
    """doubling_step (mod.rs:176-245): A = R (x, y, z Fq2) -> B = R', C = coeffs"""
    p = Prog("dbl")
    T = Tower(p)
    c, r = kernels.doubling_step(T, tuple(_fq2s(_args(p, GA, 6))))
    _rets(p, GB, [v for x in r for v in x])
    _rets(p, GC, [v for x in c for v in x])
    return p


def m_add():
    """addition_step (mod.rs:247-333): A = R, D = Q (x, y) -> B = R', C = coeffs"""
    p = Prog("add")
    T = Tower(p)
    r = tuple(_fq2s(_args(p, GA, 6)))
    qx, qy = _fq2s(_args(p, GD, 4))
    c, r2 = kernels.addition_step(T, r, qx, qy)
    _rets(p, GB, [v for x in r2 for v in x])
    _rets(p, GC, [v for x in c for v in x])
    return p


def m_ell():
    """ell (mod.rs:57-69): A = f, C = coeffs, E = P (x, y) -> B = f * line"""
    p = Prog("ell")
    T = Tower(p)
    f = _f12(_args(p, GA, 12))
    c = _fq2s(_args(p, GC, 6))
    px, py = _args(p, GE, 2)
    _rets(p, GB, _flat12(kernels.ell(T, f, c, px, py)))
    return p


def _unary12(name, fn, tower=Tower):
    def build():
        p = Prog(name)
        T = tower(p)
        _rets(p, GB, _flat12(fn(T, _f12(_args(p, GA, 12)))))
        return p
    return build


def m_mul12():
    p = Prog("mul12")
    T = Tower(p)
    a = _f12(_args(p, GA, 12))
    b = _f12(_args(p, GD, 12))
    _rets(p, GB, _flat12(T.mul12(a, b)))
    return p


MACROS = [
    ("dbl", m_dbl),
    ("add", m_add),
    ("ell", m_ell),
    ("sqr12", _unary12("sqr12", lambda T, f: T.sqr12(f))),
    ("cyc", _unary12("cyc", lambda T, f: T.cyc_sqr(f))),
    ("conj12", _unary12("conj12", lambda T, f: T.conj12(f))),
    ("mul12", m_mul12),
    ("frob1", _unary12("frob1", lambda T, f: T.frob12(f, 1))),
    ("frob2", _unary12("frob2", lambda T, f: T.frob12(f, 2))),
    ("frob3", _unary12("frob3", lambda T, f: T.frob12(f, 3))),
    ("inv12", _unary12("inv12", lambda T, f: T.inv12(f), VmTower)),
]


# ---------------- flatten / schedule / allocate ----------------
class Node:
    __slots__ = ("id", "kind", "lop", "imm", "srcs", "users", "height", "step", "slot")

    def __init__(self, id_, kind, lop, imm, srcs):
        self.id, self.kind, self.lop, self.imm, self.srcs = id_, kind, lop, imm, srcs
        self.users = []
        self.height = 0
        self.step = -1
        self.slot = None


def flatten(prog, consts, cindex):
    """The program's dataflow graph (control structure executed, variables
    turned into edges).  Sources are node ids or ("slot", ref) for constants
    (absolute slots, indexed into the shared constant table) and macro args."""
    nodes, rets = [], []
    env, vars_, counters = {}, {}, {}

    def new(kind, lop, imm, srcs):
        n = Node(len(nodes), kind, lop, imm, srcs)
        nodes.append(n)
        for s in srcs:
            if not isinstance(s, tuple):
                nodes[s].users.append(n.id)
        return n.id

    def step(op):
        k = op.kind
        s = [env[v.id] for v in op.srcs]
        if k == "const":
            key = tuple(op.imm)
            if key not in cindex:
                cindex[key] = len(consts)
                consts.append(key)
            env[op.dst.id] = ("slot", (0, cindex[key]))
        elif k == "arg":
            env[op.dst.id] = ("slot", op.imm)
        elif k == "ret":
            rets.append((op.imm, s[0]))
        elif k == "getvar":
            env[op.dst.id] = vars_[op.imm]
        elif k == "setvar":
            vars_[op.imm] = s[0]
        elif k == "sop":
            env[op.dst.id] = new(K_P2 if len(s) == 4 else K_P1, 0, None, s)
        elif k == "sqr":
            env[op.dst.id] = new(K_SQ, 0, None, s)
        elif k == "add":
            env[op.dst.id] = new(K_LIN, L_ADD, None, s)
        elif k == "sub":
            env[op.dst.id] = new(K_LIN, L_SUB, op.imm, s)
        elif k == "neg":
            env[op.dst.id] = new(K_LIN, L_NEG, op.imm, s)
        elif k == "red":
            env[op.dst.id] = new(K_LIN, L_RED, None, s)
        elif k == "inv":
            env[op.dst.id] = new(K_INV, 0, None, s)
        else:
            raise ValueError("op %s has no cooperative form" % k)

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

    run(prog.root)
    # a ret of a value that is itself an arg or constant becomes a copy (x + 0)
    for k, (ref, src) in enumerate(rets):
        if isinstance(src, tuple):
            rets[k] = (ref, new(K_LIN, L_ADD, None, [src, ("zero",)]))
    return nodes, rets


def schedule(nodes, rets):
    """List scheduling: each step takes the ready node of greatest height
    (latency-weighted path to the end) and fills the wave with the other
    ready nodes of its kind, highest first.  A node is ready once every
    source was produced by an EARLIER step."""
    for n in reversed(nodes):
        n.height = COST[n.kind] + max((nodes[u].height for u in n.users), default=0)
    pending = {n.id: sum(1 for s in n.srcs if not isinstance(s, tuple)) for n in nodes}
    ready = [n.id for n in nodes if pending[n.id] == 0]
    steps = []
    while ready:
        ready.sort(key=lambda i: (-nodes[i].height, i))
        kind = nodes[ready[0]].kind
        cap = 1 if kind == K_INV else LANES
        batch = [i for i in ready if nodes[i].kind == kind][:cap]
        taken = set(batch)
        ready = [i for i in ready if i not in taken]
        for i in batch:
            nodes[i].step = len(steps)
        steps.append((kind, batch))
        for i in batch:
            for u in nodes[i].users:
                pending[u] -= 1
                if pending[u] == 0:
                    ready.append(u)
    assert all(n.step >= 0 for n in nodes), "unscheduled nodes (cycle?)"
    return steps


def allocate(nodes, rets, steps, scratch0):
    """Slots: a returned value is written straight to its output slot (group
    B / C); other values get absolute scratch slots from scratch0 on, reused
    after their last reader (from the step after it: a LIN step's divergent
    opcodes run one after another)."""
    out_of = {}
    for ref, src in rets:
        assert src not in out_of, "value returned twice"
        out_of[src] = ref
    last = {}
    for n in nodes:
        for s in n.srcs:
            if not isinstance(s, tuple):
                last[s] = max(last.get(s, -1), n.step)
    free, top = [], scratch0
    release = {}
    for si, (kind, batch) in enumerate(steps):
        free.extend(release.pop(si, []))
        for i in batch:
            n = nodes[i]
            if i in out_of:
                n.slot = out_of[i]
                continue
            if free:
                idx = free.pop()
            else:
                idx = top
                top += 1
            n.slot = (0, idx)
            release.setdefault(last.get(i, n.step) + 1, []).append(idx)
    return top


def ref16(ref):
    g, i = ref
    assert 0 <= g < 16 and 0 <= i < 4096
    return (g << 12) | i


class Macro:
    def __init__(self, name, prog, consts, cindex):
        self.name, self.prog = name, prog
        self.nodes, self.rets = flatten(prog, consts, cindex)

    def build(self, scratch0, zero_slot):
        self.steps = schedule(self.nodes, self.rets)
        self.top = allocate(self.nodes, self.rets, self.steps, scratch0)
        self.records = []
        for kind, batch in self.steps:
            recs = []
            for i in batch:
                n = self.nodes[i]
                srcs = []
                for s in n.srcs:
                    if isinstance(s, tuple) and s[0] == "zero":
                        srcs.append(ref16((0, zero_slot)))
                    elif isinstance(s, tuple):
                        srcs.append(ref16(s[1]))
                    else:
                        srcs.append(ref16(self.nodes[s].slot))
                if kind == K_P1:
                    srcs += [ref16((0, zero_slot))] * 2
                recs.append([n.lop | ((n.imm or 0) << 4), ref16(n.slot)] + (srcs + [0] * 4)[:4])
            self.records.append((kind, recs))

    def stats(self):
        by = {}
        for kind, recs in self.records:
            c, lanes = by.get(KIND_NAME[kind], (0, 0))
            by[KIND_NAME[kind]] = (c + 1, lanes + len(recs))
        return {"nodes": len(self.nodes), "steps": len(self.records), "scratch_top": self.top, "by_kind": by,
                "est_instr": sum(COST[k] for k, _ in self.records)}


def build_all():
    consts, cindex = [], {}
    zero = tuple(dsl.to_mont_limbs(0))
    cindex[zero] = 0
    consts.append(zero)
    macros = [Macro(name, f(), consts, cindex) for name, f in MACROS]
    # the ML / FE drivers also need one (Fq12::one, R' mod q) and the INV fix-up
    # constant R'^3 mod q (bgcd gives the plain inverse)
    for extra in (dsl.to_mont_limbs(1), tuple(dsl.gen_fl.limbs(dsl.R ** 3 % dsl.Q))):
        if tuple(extra) not in cindex:
            cindex[tuple(extra)] = len(consts)
            consts.append(tuple(extra))
    scratch0 = len(consts)
    for m in macros:
        m.build(scratch0, 0)
    return macros, consts


# ---------------- replay (the GPU's semantics, in Python) ----------------
def replay(m, consts, args):
    """args: {(group, index): limbs}; returns {(group, index): limbs} of outputs"""
    V = {(0, c): tuple(v) for c, v in enumerate(consts)}
    V.update({k: tuple(v) for k, v in args.items()})

    def at(r):
        return V[(r >> 12, r & 4095)]
    for kind, recs in m.records:
        res = []
        for op, dst, a, b, c, d in recs:
            if kind in (K_P1, K_P2):
                r = dsl.mont_sop([(at(a), at(b)), (at(c), at(d))])
            elif kind == K_SQ:
                r = dsl.mont_sop([(at(a), at(a))])
            elif kind == K_INV:
                v = dsl.val_of(at(a)) % dsl.Q
                r = tuple(dsl.gen_fl.limbs(dsl.R * dsl.R * pow(v, -1, dsl.Q) % dsl.Q if v else 0))
            else:
                lop, imm = op & 15, op >> 4
                if lop == L_ADD:
                    r = tuple(x + y for x, y in zip(at(a), at(b)))
                elif lop == L_SUB:
                    r = tuple(x + ci - y for x, ci, y in zip(at(a), dsl.SUBC[imm], at(b)))
                elif lop == L_NEG:
                    r = tuple(ci - y for ci, y in zip(dsl.SUBC[imm], at(a)))
                else:
                    r = dsl.red_limbs(at(a))
            res.append(((dst >> 12, dst & 4095), r))
        for dst, r in res:      # a step's lanes all read before any writes
            V[dst] = r
    return {ref: V[ref] for ref, _ in m.rets}


def check(macros, consts, trials=3):
    rng = random.Random(11)
    for m in macros:
        groups = {}
        for n in m.prog.root.items:
            pass
        refs = set()

        def collect(block):
            for it in block.items:
                if isinstance(it, (Loop, If)):
                    collect(it.body)
                elif it.kind == "arg":
                    refs.add(it.imm)
        collect(m.prog.root)
        for _ in range(trials):
            args = {r: tuple(dsl.to_mont_limbs(rng.randrange(dsl.Q))) for r in refs}
            want = dsl.evaluate(m.prog, args)
            got = replay(m, consts, args)
            assert got == want, "%s: schedule replay differs from the DSL macro" % m.name
        del groups
    print("all %d macros: schedule replay == DSL (%d trials each)" % (len(macros), trials))


# ---------------- header ----------------
def emit(macros, consts, path):
    steps, recs, mtab = [], [], []
    for m in macros:
        mtab.append((len(steps), len(m.records)))
        for kind, rr in m.records:
            steps.append((kind, len(rr), len(recs)))
            recs.extend(rr)
    nslots = max(m.top for m in macros)
    L = ["// GENERATED by tools/pgen/coop.py -- cooperative (one wave per item) macro-operations", "#pragma once",
         "#include <stdint.h>", "namespace pa {", "namespace coop {",
         "enum : uint8_t { K_LIN = %d, K_P1, K_P2, K_SQ, K_INV };" % K_LIN,
         "enum : uint16_t { L_ADD = %d, L_SUB, L_NEG, L_RED };" % L_ADD,
         "enum Macro : int { %s, kMacros };" % ", ".join("M_%s" % m.name.upper() for m in macros),
         "constexpr int kConsts = %d;      // absolute slots 0 .. kConsts-1: constants (slot 0 = zero)" % len(consts),
         "constexpr int kZeroSlot = 0, kOneSlot = %d, kInvFixSlot = %d;" % (
             consts.index(tuple(dsl.to_mont_limbs(1))), consts.index(tuple(dsl.gen_fl.limbs(dsl.R ** 3 % dsl.Q)))),
         "constexpr int kAbsSlots = %d;    // constants + the largest macro's temporaries" % nslots,
         "constexpr int kSteps = %d, kRecords = %d;" % (len(steps), len(recs)),
         "__device__ const uint32_t kConst[%d][14] = {%s};" % (
             len(consts), ", ".join("{" + ", ".join("0x%xu" % x for x in c) + "}" for c in consts)),
         "// macro -> (first step, steps)",
         "__device__ const uint16_t kMacro[%d][2] = {%s};" % (len(mtab), ", ".join("{%d, %d}" % t for t in mtab)),
         "// step -> kind | lanes << 8, first record",
         "__device__ const uint32_t kStep[%d][2] = {%s};" % (
             len(steps), ", ".join("{%du, %du}" % (k | (n << 8), b) for k, n, b in steps)),
         "__device__ const uint16_t kRecord[%d][6] = {%s};" % (
             len(recs), ", ".join("{" + ",".join(str(x) for x in r) + "}" for r in recs)),
         "}  // namespace coop", "}  // namespace pa", ""]
    with open(path, "w") as f:
        f.write("\n".join(L))
    return len(steps), len(recs), nslots


def main():
    macros, consts = build_all()
    for m in macros:
        print("%-7s %s" % (m.name, m.stats()))
    if "--check" in sys.argv:
        check(macros, consts)
    out = os.path.join(ROOT, "pairing_amd", "csrc", "coop_prog.h")
    ns, nr, nslots = emit(macros, consts, out)
    print("wrote %s: %d steps, %d lane records (%d B), %d absolute slots, %d constants"
          % (out, ns, nr, nr * 12, nslots, len(consts)))


if __name__ == "__main__":
    main()
