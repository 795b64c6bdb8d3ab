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
# DSL-level LIN ops
L_ADD, L_SUB, L_NEG, L_RED = range(4)
# lane-level chain ops of a LIN task: acc = slot s0, then up to 4 of these
C_END, C_ADD, C_SUB, C_RSUB, C_NEG, C_RED, C_DBL = range(7)
MAX_CHAIN, MAX_SIDE = 4, 3
# latency estimates (instructions) for the list scheduler's priorities
COST = {K_LIN: 90, K_P1: 560, K_P2: 760, K_SQ: 480, K_INV: 9000}
GA, GB, GC, GD, GE, GF, GG = 1, 2, 3, 4, 5, 6, 7   # operand areas


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


def _ml_body(p, T, with_add):
    """One pipelined Miller-loop iteration (mod.rs:72-91): the f chain uses
    the coefficients c_in computed by the previous macro, while the R chain
    already computes the next doubling -- the two chains are independent, so
    the scheduler overlaps them.  A = f -> B = f', C = c_in, D = R_in,
    E = R_out, F = c_out, G = (px, py, qx.c0, qx.c1, qy.c0, qy.c1)."""
    f = _f12(_args(p, GA, 12))
    c = _fq2s(_args(p, GC, 6))
    r = tuple(_fq2s(_args(p, GD, 6)))
    px, py, qx0, qx1, qy0, qy1 = _args(p, GG, 6)
    f = kernels.ell(T, f, c, px, py)
    if with_add:
        ca, r = kernels.addition_step(T, r, (qx0, qx1), (qy0, qy1))
        f = kernels.ell(T, f, ca, px, py)
    f = T.sqr12(f)
    cd, r = kernels.doubling_step(T, r)
    _rets(p, GB, _flat12(f))
    _rets(p, GE, [v for x in r for v in x])
    _rets(p, GF, [v for x in cd for v in x])


def m_mli():
    p = Prog("mli")
    _ml_body(p, Tower(p), False)
    return p


def m_mla():
    p = Prog("mla")
    _ml_body(p, Tower(p), True)
    return p


def m_mll():
    """the final line and the conjugation (mod.rs:93-99): A = f, C = c, G = P"""
    p = Prog("mll")
    T = Tower(p)
    f = _f12(_args(p, GA, 12))
    c = _fq2s(_args(p, GC, 6))
    px, py = _args(p, GG, 2)
    _rets(p, GB, _flat12(T.conj12(kernels.ell(T, f, c, px, py))))
    return p


MACROS = [
    ("dbl", m_dbl),
    ("mli", m_mli),
    ("mla", m_mla),
    ("mll", m_mll),
    ("cyc", _unary12("cyc", lambda T, f: T.cyc_sqr(f))),
    ("conj12", _unary12("conj12", lambda T, f: T.conj12(f))),
    ("mul12", m_mul12),
    ("frob1", _unary12("frob1", lambda T, f: T.frob12(f, 1))),
    ("frob2", _unary12("frob2", lambda T, f: T.frob12(f, 2))),
    ("frob3", _unary12("frob3", lambda T, f: T.frob12(f, 3))),
    ("inv12", _unary12("inv12", lambda T, f: T.inv12(f), VmTower)),
]


# ---------------- dataflow graph ----------------
class Node:
    __slots__ = ("id", "kind", "lop", "imm", "srcs", "users", "ret")

    def __init__(self, id_, kind, lop, imm, srcs):
        self.id, self.kind, self.lop, self.imm, self.srcs = id_, kind, lop, imm, srcs
        self.users = []
        self.ret = None


def flatten(prog, consts, cindex):
    """The program's dataflow graph (control structure executed, variables
    turned into edges).  Sources are node ids or ("slot", (group, index)) for
    constants (absolute slots into the shared constant table) and args."""
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
    # a ret of an arg / constant, or of a value returned twice, becomes a copy (x + 0)
    seen = set()
    for k, (ref, src) in enumerate(rets):
        if isinstance(src, tuple) or src in seen:
            src = new(K_LIN, L_ADD, None, [src, ("slot", (0, 0))])
            rets[k] = (ref, src)
        seen.add(src)
        nodes[src].ret = ref
    return nodes, rets


# ---------------- tasks: products, INV, fused LIN chains ----------------
class Task:
    """One lane's work in one step.  PROD / INV: one node.  LIN: a chain of
    up to MAX_CHAIN LIN nodes, each consuming the previous one's value (the
    accumulator) and at most MAX_SIDE side operands in total; only the last
    node's value is materialized."""
    __slots__ = ("id", "kind", "nodes", "out", "deps", "users", "height", "step", "slot")

    def __init__(self, id_, kind, nodes_):
        self.id, self.kind, self.nodes = id_, kind, nodes_
        self.out = nodes_[-1]
        self.deps, self.users = set(), []
        self.height, self.step, self.slot = 0, -1, None


def build_tasks(nodes):
    """Fold single-use LIN values into their LIN user's chain (as its
    accumulator), left to right, so a chain of k dependent additions /
    subtractions / reductions is one lane task instead of k steps."""
    absorbed = {}          # node id -> chain root that absorbed it

    def side_srcs(n, acc):
        out, used_acc = [], False
        for s in n.srcs:
            if not used_acc and s == acc:
                used_acc = True
                continue
            out.append(s)
        return out

    chain_of = {}
    order = []
    for n in nodes:
        if n.kind != K_LIN:
            order.append([n.id])
            chain_of[n.id] = order[-1]
            continue
        # candidate accumulator: a LIN source with this node as its only user,
        # not returned, whose chain still has room
        best = None
        for s in n.srcs:
            if isinstance(s, tuple):
                continue
            m = nodes[s]
            if m.kind != K_LIN or m.ret is not None or len(m.users) != 1 or s in absorbed:
                continue
            ch = chain_of[s]
            if ch[-1] != s or len(ch) >= MAX_CHAIN:
                continue
            sides = sum(len(side_srcs(nodes[x], prev)) for x, prev in zip(ch, [None] + ch[:-1]))
            sides += len(side_srcs(n, s))
            if n.lop == L_ADD and n.srcs[0] == n.srcs[1]:
                sides -= 1                 # dbl: both operands are the accumulator
            if sides > MAX_SIDE + 1:       # the head may read two slots
                continue
            if best is None or len(chain_of[s]) > len(chain_of[best]):
                best = s
        if best is not None:
            ch = chain_of[best]
            ch.append(n.id)
            absorbed[best] = n.id
            chain_of[n.id] = ch
        else:
            order.append([n.id])
            chain_of[n.id] = order[-1]
    tasks = []
    owner = {}
    for ch in order:
        t = Task(len(tasks), nodes[ch[0]].kind, ch)
        tasks.append(t)
        for x in ch:
            owner[x] = t.id
    for t in tasks:
        inner = set(t.nodes)
        for x in t.nodes:
            for s in nodes[x].srcs:
                if not isinstance(s, tuple) and s not in inner:
                    t.deps.add(owner[s])
        for d in t.deps:
            tasks[d].users.append(t.id)
    return tasks, owner


def schedule(tasks):
    """List scheduling over tasks.  Products of any form share a step (the
    step runs the sop2 leaf, P1 lanes padding with zero, unless every lane is
    a plain product / square).  The step kind is that of the ready task of
    greatest height; a product step is postponed while a LIN task that leads
    to a product of (almost) the same height is still ready, so products of
    one level meet in one step."""
    def cost(t):
        return COST[K_P2 if t.kind in (K_P1, K_P2, K_SQ) else t.kind] if t.kind != K_LIN else \
            COST[K_LIN] + 25 * len(t.nodes)
    for t in reversed(tasks):
        t.height = cost(t) + max((tasks[u].height for u in t.users), default=0)
    pending = {t.id: len(t.deps) for t in tasks}
    ready = [t.id for t in tasks if not t.deps]
    steps = []
    prod = (K_P1, K_P2, K_SQ)
    while ready:
        ready.sort(key=lambda i: (-tasks[i].height, i))
        top = tasks[ready[0]]
        cls = "P" if top.kind in prod else top.kind
        if cls == "P":
            best_lin = max((tasks[i].height for i in ready if tasks[i].kind == K_LIN), default=-1)
            if best_lin > top.height - COST[K_P2] // 2:
                cls = K_LIN
        if cls == "P":
            batch = [i for i in ready if tasks[i].kind in prod][:LANES]
            kinds = {tasks[i].kind for i in batch}
            kind = K_SQ if kinds == {K_SQ} else (K_P2 if K_P2 in kinds else K_P1)
        else:
            cap = 1 if cls == K_INV else LANES
            batch = [i for i in ready if tasks[i].kind == cls][:cap]
            kind = cls
        taken = set(batch)
        ready = [i for i in ready if i not in taken]
        for i in batch:
            tasks[i].step = len(steps)
        steps.append((kind, batch))
        for i in batch:
            for u in tasks[i].users:
                pending[u] -= 1
                if pending[u] == 0:
                    ready.append(u)
    assert all(t.step >= 0 for t in tasks), "unscheduled tasks (cycle?)"
    return steps


def allocate(nodes, tasks, steps, scratch0):
    """Slots: a returned value is written straight to its output slot;
    other task outputs get absolute scratch slots from scratch0 on, reused
    after their last reader (from the step after it: a LIN step's divergent
    chain opcodes run one after another)."""
    last = {}
    for t in tasks:
        for d in t.deps:
            last[d] = max(last.get(d, -1), t.step)
    free, top = [], scratch0
    release = {}
    for si, (kind, batch) in enumerate(steps):
        free.extend(release.pop(si, []))
        for i in batch:
            t = tasks[i]
            ref = nodes[t.out].ret
            if ref is not None:
                t.slot = ref
                continue
            if free:
                idx = free.pop()
            else:
                idx = top
                top += 1
            t.slot = (0, idx)
            release.setdefault(last.get(i, t.step) + 1, []).append(idx)
    return top


def ref16(ref):
    g, i = ref
    assert 0 <= g < 8 and 0 <= i < 8192
    return (g << 13) | i


class Macro:
    def __init__(self, name, prog, consts, cindex):
        self.name, self.prog = name, prog
        self.nodes, self.rets = flatten(prog, consts, cindex)

    def build(self, scratch0):
        nodes = self.nodes
        self.tasks, owner = build_tasks(nodes)
        self.steps = schedule(self.tasks)
        self.top = allocate(nodes, self.tasks, self.steps, scratch0)
        tasks = self.tasks

        def src_ref(s):
            if isinstance(s, tuple):
                return ref16(s[1])
            return ref16(tasks[owner[s]].slot)
        self.records = []
        for kind, batch in self.steps:
            recs = []
            for i in batch:
                t = tasks[i]
                dst = ref16(t.slot)
                if kind in (K_P1, K_P2, K_SQ):
                    n = nodes[t.out]
                    srcs = [src_ref(x) for x in n.srcs]
                    if n.kind == K_SQ:
                        srcs = srcs * 2                           # a * a
                    if len(srcs) == 2:
                        srcs += [ref16((0, 0))] * 2               # + 0 * 0
                    recs.append([0, dst] + srcs + [0, 0])
                elif kind == K_INV:
                    recs.append([0, dst, src_ref(nodes[t.out].srcs[0]), 0, 0, 0, 0, 0])
                else:
                    recs.append(self._chain(t, src_ref, dst))
            self.records.append((kind, recs))

    def _chain(self, t, src_ref, dst):
        """LIN task -> [nops, dst, s0, s1, s2, s3, ops01, ops23]: acc = s0,
        then op j (8 bits: code | bound << 3) taking the next side slot"""
        nodes = self.nodes
        ops, slots = [], []
        acc = None
        for x in t.nodes:
            n = nodes[x]
            srcs = list(n.srcs)
            if acc is None:
                # head: load the first operand into the accumulator
                first = srcs[0]
                slots.append(src_ref(first))
                acc_src = first
            else:
                acc_src = acc
            rest = list(srcs)
            rest.remove(acc_src)
            if n.lop == L_ADD:
                if rest == [acc_src]:
                    ops.append((C_DBL, 0))
                else:
                    ops.append((C_ADD, 0))
                    slots.append(src_ref(rest[0]))
            elif n.lop == L_SUB:
                if srcs[0] == acc_src and srcs[0] != srcs[1]:
                    ops.append((C_SUB, n.imm))        # acc - x, x of bound imm
                    slots.append(src_ref(srcs[1]))
                elif srcs[1] == acc_src and srcs[0] != srcs[1]:
                    ops.append((C_RSUB, n.imm))       # x - acc, acc of bound imm
                    slots.append(src_ref(srcs[0]))
                else:
                    raise AssertionError("a - a in a chain")
            elif n.lop == L_NEG:
                ops.append((C_NEG, n.imm))
            else:
                ops.append((C_RED, 0))
            acc = x
        assert len(ops) <= MAX_CHAIN and len(slots) <= 1 + MAX_SIDE, (ops, slots)
        packed = [code | (imm << 3) for code, imm in ops] + [0] * (4 - len(ops))
        assert all(p < 256 for p in packed)
        slots += [0] * (4 - len(slots))
        return [len(ops), dst] + slots + [packed[0] | packed[1] << 8, packed[2] | packed[3] << 8]

    def stats(self):
        by = {}
        for kind, recs in self.records:
            c, lanes = by.get(KIND_NAME[kind], (0, 0))
            by[KIND_NAME[kind]] = (c + 1, lanes + len(recs))
        est = sum(COST[k] + (25 * max(r[0] for r in recs) if k == K_LIN else 0) for k, recs in self.records)
        return {"nodes": len(self.nodes), "tasks": len(self.tasks), "steps": len(self.records),
                "scratch_top": self.top, "by_kind": by, "est_instr": est}


def build_all():
    consts, cindex = [], {}
    zero = tuple(dsl.to_mont_limbs(0))
    cindex[zero] = 0
    consts.append(zero)
    macros = [Macro(name, f(), consts, cindex) for name, f in MACROS]
    # the drivers also need one (Fq12::one, R' mod q) and the INV fix-up
    # constant R'^3 mod q (bgcd gives the plain inverse)
    for extra in (dsl.to_mont_limbs(1), tuple(dsl.gen_fl.limbs(dsl.R ** 3 % dsl.Q))):
        if tuple(extra) not in cindex:
            cindex[tuple(extra)] = len(consts)
            consts.append(tuple(extra))
    scratch0 = len(consts)
    for m in macros:
        m.build(scratch0)
    return macros, consts


# ---------------- replay (the GPU's semantics, in Python) ----------------
def replay(m, consts, args):
    """args: {(group, index): limbs}; returns {(group, index): limbs} of outputs"""
    V = {(0, c): tuple(v) for c, v in enumerate(consts)}
    V.update({k: tuple(v) for k, v in args.items()})

    def at(r):
        return V[(r >> 13, r & 8191)]
    for kind, recs in m.records:
        res = []
        for rec in recs:
            hdr, dst, a, b, c, d, o01, o23 = rec
            if kind in (K_P1, K_P2):
                r = dsl.mont_sop([(at(a), at(b)), (at(c), at(d))])
            elif kind == K_SQ:
                r = dsl.mont_sop([(at(a), at(a))])
            elif kind == K_INV:
                v = dsl.val_of(at(a)) % dsl.Q
                r = tuple(dsl.gen_fl.limbs(dsl.R * dsl.R * pow(v, -1, dsl.Q) % dsl.Q if v else 0))
            else:
                acc = at(a)
                side = [b, c, d]
                packed = [o01 & 255, o01 >> 8, o23 & 255, o23 >> 8]
                for j in range(hdr):
                    code, imm = packed[j] & 7, packed[j] >> 3
                    if code == C_ADD:
                        acc = tuple(x + y for x, y in zip(acc, at(side.pop(0))))
                    elif code == C_DBL:
                        acc = tuple(x + x for x in acc)
                    elif code == C_SUB:
                        acc = tuple(x + ci - y for x, ci, y in zip(acc, dsl.SUBC[imm], at(side.pop(0))))
                    elif code == C_RSUB:
                        acc = tuple(y + ci - x for x, ci, y in zip(acc, dsl.SUBC[imm], at(side.pop(0))))
                    elif code == C_NEG:
                        acc = tuple(ci - x for x, ci in zip(acc, dsl.SUBC[imm]))
                    elif code == C_RED:
                        acc = dsl.red_limbs(acc)
                    else:
                        raise AssertionError(code)
                r = acc
            res.append(((dst >> 13, dst & 8191), r))
        for dst, r in res:      # a step's lanes all read before any writes
            V[dst] = r
    return {ref: V[ref] for ref, _ in m.rets}


def check(macros, consts, trials=3):
    rng = random.Random(11)
    for m in macros:
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
         "enum : uint32_t { C_END = %d, C_ADD, C_SUB, C_RSUB, C_NEG, C_RED, C_DBL };" % C_END,
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
         "// record: hdr (LIN: chain length), dst, s0..s3, chain ops 0|1, 2|3 (code | bound << 3)",
         "__device__ const uint16_t kRecord[%d][8] = {%s};" % (
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
          % (out, ns, nr, nr * 16, nslots, len(consts)))


if __name__ == "__main__":
    main()
