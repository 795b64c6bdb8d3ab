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
K_LIN, K_P1, K_P2, K_SQ, K_INV, K_LC = range(6)
KIND_NAME = ["LIN", "P1", "P2", "SQ", "INV", "LC"]
# LC (linear combination) tasks replace the LIN chains unless COOP_CHAINS=1:
# every LIN subgraph between products collapses to sum c_i x_i over
# materialized values (products, inversions, arguments, constants), one lane
# task per product operand / returned value, so the steps between two
# product levels are one LC step instead of a LIN level per chain depth.
LC = os.environ.get("COOP_CHAINS", "0") != "1"
LC_TMAX = 15       # terms of one LC task (incl. the zero padding of a split)
# macros whose product lanes compute their <= 2-term operands in a prologue
# (one-wave VM: a wash on the Miller-loop macros, -5 % on the cyclotomic
# square; quad VM (profiles/r03_s3_coop_pairs_ab.txt): ML +13 % with
# prologues, FE -3 % with them on every FE macro)
PAIRS = set(os.environ.get("COOP_PAIRS", "cyc,conj12,mul12,frob1,frob2,frob3,inv12").split(","))
SPLIT_SOP = os.environ.get("COOP_SPLIT_SOP", "1") == "1"   # measured: +2.5k cycles per product step, a wash
# DSL-level LIN ops
L_ADD, L_SUB, L_NEG, L_RED = range(4)
# lane-level chain ops of a LIN task: acc = slot s0, then up to 4 of these
C_END, C_ADD, C_SUB, C_RSUB, C_NEG, C_RED, C_DBL = range(7)
MAX_CHAIN, MAX_SIDE = 4, 3
# latency estimates (instructions) for the list scheduler's priorities
COST = {K_LIN: 90, K_P1: 560, K_P2: 760, K_SQ: 480, K_INV: 9000, K_LC: 60}
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
    __slots__ = ("id", "kind", "nodes", "out", "deps", "users", "height", "step", "slot", "form", "red", "opnd", "u",
                 "lay")

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


def form_u(f):
    """limb bound U of sum c x over F<1> leaves: the positive part plus the
    subtraction constant C_B, B = sum of the negative coefficients (99: none fits)"""
    pos = sum(c for c in f.values() if c > 0)
    neg = -sum(c for c in f.values() if c < 0)
    if neg > 14:
        return 99
    return pos + (dsl.SUBCU[neg] if neg else 0)


def lc_layout(form, split):
    """term order of an LC task for a step whose lanes reduce (red) their
    partial sum after `split` terms (0: no mid-step reduction): the first
    segment keeps U <= 16; the reduced value (F<1>) plus C_B2 plus the rest
    too.  Largest coefficients first; the first segment is padded to `split`
    with (zero slot, 0).  None if the form does not fit."""
    items = sorted(form.items(), key=lambda kv: (-abs(kv[1]), kv[0]))
    if not split:
        return items if len(items) <= LC_TMAX and form_u(dict(items)) <= 16 else None
    seg1, rest = [], []
    for kv in items:
        if len(seg1) < split and form_u(dict(seg1 + [kv])) <= 16:
            seg1.append(kv)
        else:
            rest.append(kv)
    neg2 = -sum(c for _, c in rest if c < 0)
    if neg2 > 14 or 1 + form_u(dict(rest)) > 16 or split + len(rest) > LC_TMAX:
        return None
    return seg1 + [(("s", (0, 0)), 0)] * (split - len(seg1)) + rest


def lc_fits(form):
    return any(lc_layout(form, sp) is not None for sp in (0, 4, 8))


def lc_forms(nodes, mat):
    """LIN node -> {leaf: coefficient}; leaves are ("n", id) for products,
    inversions and materialized LIN nodes, ("s", slot) for arguments and
    constants (the zero constant dropped).  red is the identity on values."""
    form = {}

    def get(x):
        if isinstance(x, tuple):
            return {} if x[1] == (0, 0) else {("s", x[1]): 1}
        if nodes[x].kind != K_LIN or x in mat:
            return {("n", x): 1}
        return form[x]
    for n in nodes:
        if n.kind != K_LIN:
            continue
        f = dict(get(n.srcs[0]))
        if n.lop == L_ADD:
            for k, v in get(n.srcs[1]).items():
                f[k] = f.get(k, 0) + v
        elif n.lop == L_SUB:
            for k, v in get(n.srcs[1]).items():
                f[k] = f.get(k, 0) - v
        elif n.lop == L_NEG:
            f = {k: -v for k, v in f.items()}
        form[n.id] = {k: v for k, v in f.items() if v}
    return form, get


def build_lc_tasks(nodes, pairs=False):
    """Tasks for the LC form: products / inversions as before, and one LC
    task per LIN value that is a product or inversion operand (unless it is a
    bare leaf), a returned value, or materialized because a form using it
    would exceed LC_TMAX terms or the bound U <= 16."""
    prod = (K_P1, K_P2, K_SQ)
    mat = set()
    while True:
        form, get = lc_forms(nodes, mat)
        need = set(mat)
        for n in nodes:
            if n.kind in prod or n.kind == K_INV:
                need |= {x for x in n.srcs if not isinstance(x, tuple) and nodes[x].kind == K_LIN}
            if n.ret is not None and n.kind == K_LIN:
                need.add(n.id)
        bad = [x for x in sorted(need) if not lc_fits(form[x])]
        if not bad:
            break
        grew = len(mat)
        for x in bad:
            # materialize the unmaterialized LIN source with the biggest form
            # (none left: a source was materialized for an earlier one this round)
            kids = [y for y in nodes[x].srcs if not isinstance(y, tuple) and nodes[y].kind == K_LIN
                    and y not in mat]
            if kids:
                mat.add(max(kids, key=lambda y: (len(form[y]), form_u(form[y]), y)))
        assert len(mat) > grew, "LC forms too big with leaf sources only: %s" % bad
    # tasks, in node order
    tasks, owner = [], {}
    # a returned LIN value that is one F<1> leaf (a product, an inversion or a
    # materialized value, coefficient 1) is returned by that leaf's task
    # directly instead of through a copy step
    for x in sorted(need):
        n = nodes[x]
        f = form[x]
        if n.ret is None or x in mat or len(f) != 1 or \
                any(x in nodes[u].srcs for u in n.users if nodes[u].kind != K_LIN):
            continue
        (k, c), = f.items()
        if c != 1 or k[0] != "n" or nodes[k[1]].ret is not None:
            continue
        y = k[1]
        if nodes[y].kind == K_LIN and y not in mat:
            continue
        nodes[y].ret, n.ret = n.ret, None
        need.discard(x)
    lc_nodes = sorted(need)
    lcset = set(lc_nodes)
    for n in nodes:
        if n.kind in prod or n.kind == K_INV or n.id in lcset:
            t = Task(len(tasks), n.kind if n.id not in lcset else K_LC, [n.id])
            t.form = sorted(form[n.id].items()) if n.id in lcset else None
            t.red = n.id in lcset and (n.id in mat or n.ret is not None)
            t.opnd = None
            tasks.append(t)
            owner[n.id] = t.id
    # product operands: a bare leaf (one term, coefficient 1), a "pair" -- at
    # most two terms, computed in the product lane's prologue (COOP_PAIRS) --
    # or an LC task; a bare-leaf LC task not returned / materialized is dropped
    def leafref(k):
        return ("s", k[1]) if k[0] == "s" else ("t", owner[k[1]])

    def ref_of(x, pairs_ok):
        """operand x of a product / inversion -> ("t", task), ("s", slot) or
        ("p", terms, U, node)"""
        if isinstance(x, tuple):
            return ("s", x[1])
        if nodes[x].kind == K_LIN and not tasks[owner[x]].red:
            f = form[x]
            if not f:
                return ("s", (0, 0))
            if len(f) == 1:
                (k, c), = f.items()
                if c == 1:
                    return leafref(k)
            if pairs_ok and pairs and len(f) <= 2 and form_u(f) <= 4:
                return ("p", tuple((leafref(k), c) for k, c in sorted(f.items())), form_u(f), x)
        return ("t", owner[x])
    for t in tasks:
        if t.kind == K_LC:
            t.u = 1 if t.red else form_u(dict(t.form))
        elif t.kind in prod or t.kind == K_INV:
            t.opnd = [ref_of(x, t.kind != K_INV) for x in nodes[t.out].srcs]

    # red the largest operand (a pair becomes its LC task first) until every
    # product's column bound holds (P1 / P2: sum U_a U_b <= 17, SQ: U <= 2)
    def u_of(r):
        if r[0] == "p":
            return r[2]
        return tasks[r[1]].u if r[0] == "t" and tasks[r[1]].kind == K_LC else 1
    for t in tasks:
        if t.kind not in prod and t.kind != K_INV:
            continue
        while True:
            us = [u_of(r) for r in t.opnd]
            if t.kind == K_INV:
                ok = us[0] == 1
            elif t.kind == K_SQ:
                ok = us[0] <= 2
            else:
                ok = sum(us[2 * k] * us[2 * k + 1] for k in range(len(us) // 2)) <= 17
            if ok:
                break
            k = max(range(len(us)), key=lambda j: (us[j], j))
            r = t.opnd[k]
            if r[0] == "p":
                t.opnd[k] = ("t", owner[r[3]])
            else:
                assert r[0] == "t" and tasks[r[1]].kind == K_LC and tasks[r[1]].u > 1
                tasks[r[1]].red, tasks[r[1]].u = True, 1
    used = set()
    for t in tasks:
        for r in t.opnd or ():
            if r[0] == "t":
                used.add(r[1])
            elif r[0] == "p":
                used |= {lr[1] for lr, _ in r[1] if lr[0] == "t"}
    keep = [t for t in tasks if t.kind != K_LC or t.red or t.id in used]
    # renumber, dependencies
    remap = {t.id: k for k, t in enumerate(keep)}
    for k, t in enumerate(keep):
        t.id = k
        t.deps, t.users = set(), []
    for t in keep:
        if t.kind == K_LC:
            t.deps = {remap[owner[k[1]]] for k, _ in t.form if k[0] == "n"}
        else:
            def rm(r):
                if r[0] == "t":
                    return ("t", remap[r[1]])
                if r[0] == "p":
                    return ("p", tuple((rm(lr), c) for lr, c in r[1]), r[2], r[3])
                return r
            t.opnd = [rm(r) for r in t.opnd]
            t.deps = {r[1] for r in t.opnd if r[0] == "t"} | \
                {lr[1] for r in t.opnd if r[0] == "p" for lr, _ in r[1] if lr[0] == "t"}
        for d in t.deps:
            keep[d].users.append(t.id)
    owner2 = {t.out: t.id for t in keep}
    return keep, owner2


def schedule(tasks):
    """List scheduling over tasks.  Products of any form share a step (the
    step runs the sop2 leaf, P1 lanes padding with zero, unless every lane is
    a plain product / square).  The step kind is that of the ready task of
    greatest height; a product step is postponed while a LIN task that leads
    to a product of (almost) the same height is still ready, so products of
    one level meet in one step."""
    def cost(t):
        if t.kind == K_LC:
            return COST[K_LC] + 25 * len(t.form) + (70 if t.red else 0)
        return COST[K_P2 if t.kind in (K_P1, K_P2, K_SQ) else t.kind] if t.kind != K_LIN else \
            COST[K_LIN] + 25 * len(t.nodes)
    # heights in reverse topological order (task ids need not be topological:
    # split products are appended after their users)
    order, indeg = [], {t.id: len(t.deps) for t in tasks}
    stack = [t.id for t in tasks if not t.deps]
    while stack:
        i = stack.pop()
        order.append(i)
        for u in tasks[i].users:
            indeg[u] -= 1
            if indeg[u] == 0:
                stack.append(u)
    assert len(order) == len(tasks), "cycle in the task graph"
    for i in reversed(order):
        t = tasks[i]
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
            best_lin = max((tasks[i].height for i in ready if tasks[i].kind in (K_LIN, K_LC)), default=-1)
            if best_lin > top.height - COST[K_P2] // 2:
                cls = K_LC if LC else K_LIN
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
        if LC:
            return self.build_lc(scratch0)
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

    def build_lc(self, scratch0):
        """records of the LC form.  Products: [0, dst, a, b, c, d, 0, 0];
        LC: [nterms | red << 5 | B1 << 6 | B2 << 10, dst, (slot, coef) x
        nterms]; B1 / B2 = the sums of the negative coefficients before / after
        the step's split point (C_B added at each segment's start, 0: none)"""
        nodes = self.nodes
        self.tasks, owner = build_lc_tasks(nodes, self.name in PAIRS)
        self.steps = schedule(self.tasks)
        if SPLIT_SOP:
            # a product step whose lanes are mostly plain products runs the
            # sum-of-products leaf for all of them: split its few a*b + c*d
            # into two plain products (the sum moves into the consumers' LC
            # forms) when the lanes allow, then rebuild
            split = []
            for kind, batch in self.steps:
                if kind != K_P2:
                    continue
                two = [self.tasks[i].out for i in batch if nodes[self.tasks[i].out].kind == K_P2]
                if 4 * len(two) <= len(batch) and len(batch) + len(two) <= LANES:
                    split += two
            if split:
                for x in split:
                    self._split_sop(x)
                self.tasks, owner = build_lc_tasks(nodes, self.name in PAIRS)
                self.steps = schedule(self.tasks)
        self.top = allocate(nodes, self.tasks, self.steps, scratch0)
        tasks = self.tasks

        def ref(r):
            return ref16(r[1]) if r[0] == "s" else ref16(tasks[r[1]].slot)
        self.records = []
        self.splits = []
        self.pro = []
        for kind, batch in self.steps:
            recs = []
            split = 0
            if kind == K_LC:
                # one mid-step reduction point for the whole step (0, 4 or 8 terms)
                for split in (0, 4, 8):
                    lays = [lc_layout(dict(tasks[i].form), split) for i in batch]
                    if all(l is not None for l in lays):
                        break
                else:
                    raise AssertionError("%s: no common split for an LC step" % self.name)
                for i, l in zip(batch, lays):
                    t = tasks[i]
                    t.lay = l
                    rest = l[split:] if split else []
                    if not t.red and split and len(l) > split and 1 + form_u(dict(rest)) > t.u:
                        t.red = True       # keep the bound the products were checked with
            self.splits.append(split)
            pro = kind in (K_P1, K_P2, K_SQ) and any(r[0] == "p" for i in batch for r in tasks[i].opnd)
            self.pro.append(pro)
            for i in batch:
                t = tasks[i]
                dst = ref16(t.slot)
                if kind in (K_P1, K_P2, K_SQ) and pro:
                    # [B_a | B_b << 4 | B_c << 8 | B_d << 12, dst, a1, a2, b1, b2, c1, c2,
                    #  d1, d2, coefs a, b, c, d (two int8 each), 0, 0]: operand =
                    # C_B + x1 c1 + x2 c2
                    ops = list(t.opnd)
                    if nodes[t.out].kind == K_SQ:
                        ops = ops * 2
                    ops += [("s", (0, 0))] * (4 - len(ops))
                    flags, sl, cw = 0, [], []
                    for k, r in enumerate(ops):
                        terms = r[1] if r[0] == "p" else ((r, 1),)
                        terms = list(terms) + [(("s", (0, 0)), 0)] * (2 - len(terms))
                        flags |= (-sum(c for _, c in terms if c < 0)) << (4 * k)
                        sl += [ref(lr) for lr, _ in terms]
                        cw.append((terms[0][1] & 0xff) | (terms[1][1] & 0xff) << 8)
                    recs.append([flags, dst] + sl + cw + [0, 0])
                elif kind in (K_P1, K_P2, K_SQ):
                    srcs = [ref(r) for r in t.opnd]
                    if nodes[t.out].kind == K_SQ:
                        srcs = srcs * 2
                    if len(srcs) == 2:
                        srcs += [ref16((0, 0))] * 2
                    recs.append([0, dst] + srcs + [0, 0])
                elif kind == K_INV:
                    recs.append([0, dst, ref(t.opnd[0]), 0, 0, 0, 0, 0])
                else:
                    lay = t.lay
                    sp = split
                    seg1, seg2 = (lay[:sp], lay[sp:]) if sp else (lay, [])
                    b1 = -sum(c for _, c in seg1 if c < 0)
                    b2 = -sum(c for _, c in seg2 if c < 0)
                    rec = [len(lay) | (int(t.red) << 5) | (b1 << 6) | (b2 << 10), dst]
                    for (k, c) in lay:
                        leaf = ref16(k[1]) if k[0] == "s" else ref16(tasks[owner[k[1]]].slot)
                        rec += [leaf, c & 0xffff]
                    recs.append(rec)
            self.records.append((kind, recs))

    def _split_sop(self, x):
        """node x = a*b + c*d -> x = n1 + n2 (LIN) with n1 = a*b, n2 = c*d"""
        nodes = self.nodes
        n = nodes[x]
        a, b, c, d = n.srcs
        halves = []
        for srcs in ((a, b), (c, d)):
            h = Node(len(nodes), K_P1, 0, None, list(srcs))
            nodes.append(h)
            for s_ in srcs:
                if not isinstance(s_, tuple):
                    us = nodes[s_].users
                    if x in us:
                        us.remove(x)
                    us.append(h.id)
            h.users = [x]
            halves.append(h.id)
        n.kind, n.lop, n.imm, n.srcs = K_LIN, L_ADD, None, halves

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
        est = sum(COST[k] + (25 * max(r[0] & 31 for r in recs) if k in (K_LIN, K_LC) else 0)
                  for k, recs in self.records)
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
    for si, (kind, recs) in enumerate(m.records):
        res = []
        for rec in recs:
            if kind == K_LC:
                # the kernel's u32 limb arithmetic, checked against the F<U> contract
                nt, red, b1, b2 = rec[0] & 31, (rec[0] >> 5) & 1, (rec[0] >> 6) & 15, rec[0] >> 10
                split = m.splits[si]
                terms = [(rec[2 + 2 * j], (rec[3 + 2 * j] ^ 0x8000) - 0x8000) for j in range(nt)]
                segs = [terms[:split], terms[split:]] if split else [terms]
                acc, base_u = [0] * 14, 0
                for k, seg in enumerate(segs):
                    b = b1 if k == 0 else b2
                    assert b == -sum(c for _, c in seg if c < 0)
                    if b:
                        acc = [p + q for p, q in zip(acc, dsl.SUBC[b])]
                    for slot, cf in seg:
                        x = at(slot)
                        assert max(x) < (1 << 28) and dsl.val_of(x) < 2 * dsl.Q, "LC leaf beyond F<1>"
                        acc = [p + cf * q for p, q in zip(acc, x)]
                    u = base_u + form_u({j: c for j, (_, c) in enumerate(seg)})
                    assert all(0 <= v <= u * dsl.MASK for v in acc), "LC limbs beyond F<%d>" % u
                    if k + 1 < len(segs):
                        acc, base_u = list(dsl.red_limbs(acc)), 1
                r = dsl.red_limbs(acc) if red else tuple(acc)
                res.append(((rec[1] >> 13, rec[1] & 8191), r))
                continue
            if kind in (K_P1, K_P2, K_SQ) and len(rec) == 16:
                ops = []
                for k in range(4):
                    b = (rec[0] >> (4 * k)) & 15
                    cw = rec[10 + k]
                    cs = [((cw & 0xff) ^ 0x80) - 0x80, ((cw >> 8) ^ 0x80) - 0x80]
                    acc = list(dsl.SUBC[b]) if b else [0] * 14
                    plain = cs == [1, 0]      # a bare operand (any bound; the product checks its columns)
                    for slot, cf in zip(rec[2 + 2 * k:4 + 2 * k], cs):
                        x = at(slot)
                        if cf and not plain:
                            assert max(x) < (1 << 28) and dsl.val_of(x) < 2 * dsl.Q, "pair term beyond F<1>"
                        acc = [p + cf * q for p, q in zip(acc, x)]
                    u = form_u({j: c for j, c in enumerate(cs) if c})
                    assert plain or all(0 <= v <= u * dsl.MASK for v in acc), "prologue limbs beyond F<%d>" % u
                    ops.append(tuple(acc))
                if kind == K_SQ:
                    r = dsl.mont_sop([(ops[0], ops[0])])
                else:
                    r = dsl.mont_sop([(ops[0], ops[1]), (ops[2], ops[3])])
                res.append(((rec[1] >> 13, rec[1] & 8191), r))
                continue
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
            if LC:
                # the same field values, every output F<1> (limbs < 2^28, value < 2q)
                assert set(got) == set(want)
                for k in want:
                    assert dsl.val_of(got[k]) % dsl.Q == dsl.val_of(want[k]) % dsl.Q, \
                        "%s: LC schedule replay differs from the DSL macro at %s" % (m.name, k)
                    assert max(got[k]) < (1 << 28) and dsl.val_of(got[k]) < 2 * dsl.Q, "%s: output not F<1>" % m.name
            else:
                assert got == want, "%s: schedule replay differs from the DSL macro" % m.name
    print("all %d macros: schedule replay == DSL (%d trials each)" % (len(macros), trials))


# ---------------- header ----------------
def emit(macros, consts, path):
    steps, recs, mtab = [], [], []
    for m in macros:
        mtab.append((len(steps), len(m.records)))
        for si, (kind, rr) in enumerate(m.records):
            if kind == K_LC:
                # R rows of 8 u16 per lane (word 0 = hdr | dst, 1 + j = term j)
                T = max(r[0] & 31 for r in rr)
                R = (2 + 2 * T + 7) // 8
                assert T <= 15 and R <= 4
                steps.append((kind | (R | T << 4 | (m.splits[si] // 4) << 8) << 16, len(rr), len(recs)))
                for r in rr:
                    r = r + [0] * (8 * R - len(r))
                    recs.extend(r[8 * k:8 * k + 8] for k in range(R))
            elif kind in (K_P1, K_P2, K_SQ) and m.pro[si]:
                steps.append((kind | 2 << 16, len(rr), len(recs)))   # 2 record rows: prologue operands
                for r in rr:
                    recs.extend([r[0:8], r[8:16]])
            else:
                steps.append((kind | 1 << 16, len(rr), len(recs)))
                recs.extend(rr)
    nslots = max(m.top for m in macros)
    L = ["// GENERATED by tools/pgen/coop.py -- cooperative (one wave per item) macro-operations", "#pragma once",
         "#include <stdint.h>", "namespace pa {", "namespace coop {",
         "enum : uint8_t { K_LIN = %d, K_P1, K_P2, K_SQ, K_INV, K_LC };" % K_LIN,
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
         "// step -> kind | lanes << 8 (| LC: record rows R << 16 | max terms T << 20), first record",
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
    out = os.environ.get("COOP_OUT") or os.path.join(ROOT, "pairing_amd", "csrc", "coop_prog.h")
    ns, nr, nslots = emit(macros, consts, out)
    print("wrote %s: %d steps, %d lane records (%d B), %d absolute slots, %d constants"
          % (out, ns, nr, nr * 16, nslots, len(consts)))


if __name__ == "__main__":
    main()
