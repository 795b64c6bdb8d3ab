"""Lane-exchange ops (sel / swap / dppadd / neg / sub / add) of a lane-pair
program counted by the Tower2 method that created them, weighted by how
often the DSL trace runs them (one lane of one pairing).  DESIGN.md section 5
"Round 6".  Usage: python3 tools/pgen/exchange_sites.py fe2|ml2p"""
import sys, os, random, collections
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE); sys.path.insert(0, os.path.dirname(HERE))
import dsl, tower2, kernels
site = []
op_site = {}
orig_op = dsl.Prog._op
def _op(self, kind, srcs, u, imm=None, vb=None):
    v = orig_op(self, kind, srcs, u, imm, vb)
    if v is not None:
        op_site[v.id] = (site[-1] if site else "-", kind)
    return v
dsl.Prog._op = _op
def wrap(cls, name):
    f = getattr(cls, name)
    def g(self, *a, **k):
        site.append(name)
        try: return f(self, *a, **k)
        finally: site.pop()
    setattr(cls, name, g)
for n in ("_pair_direct", "sqr2", "xi", "conj2", "const2", "kdec_numden", "inv2", "mul2", "pair"):
    wrap(tower2.Tower2, n)
which = sys.argv[1]
if which == "fe2":
    progf = tower2.two_pass(lambda: kernels.final_exp_prog(lanes=2)); nin = 12
else:
    progf = tower2.two_pass(lambda: kernels.miller_loop_prog(lanes=2, pairing_only=True), xi_dpp=False); nin = 6
op_site.clear()
prog = progf()
rng = random.Random(1)
ins = {k: rng.randrange(dsl.Q) for k in range(nin)}
tr = []
dsl.evaluate(prog, ins, None, tr)
cnt = collections.Counter()
for vid, r, op in tr:
    s = op_site.get(vid, ("?", op.kind))
    if op.kind in ("sel", "swap", "dppadd", "neg", "sub", "add"):
        cnt[(s[0], op.kind)] += 1
for k, v in sorted(cnt.items(), key=lambda x: -x[1]):
    print("%-14s %-8s %6d" % (k[0], k[1], v))
