"""Register allocation and gfx950 instruction emission for DSL programs.

Storage model (one pairing per lane, one wave per SIMD, 512 registers):
  VGPR  v0..v15   work area of the product / reduction / record I/O code:
                  acc = v[0:1], Montgomery digits m_0..m_13 = v2..v15
        v16       tid * 8 (LDS / spill lane offset)      v17  spare
        v18..v255 17 "V slots" of 14 VGPRs, where every operand must be
  AGPR  a0..a251  18 "A slots" (VALU cannot read AGPRs: 14 accvgpr moves)
  LDS   11 "L slots" per wave, layout [slot][pair][lane] x 8 B (ds_*_b64)
  HBM   "M slots" in a per-wave workspace, same layout (global_*_dwordx2)
  SGPR  s[80:93] q limbs, s94 -q^-1 mod 2^28, s95 floor(2^400/q)

A value lives in one or more locations; operations need their sources in
V slots and define their destination in a V slot.  Within a straight-line
block the allocator evicts the V-resident value whose next use is furthest
(Belady), dropping it if a copy exists elsewhere (a variable's home, an
earlier spill) and otherwise spilling to an A, then L, then M slot.
Variables (DSL getvar/setvar) have fixed homes for their lifetime; values
that live across a loop / branch are parked in A/L/M slots the body does
not touch.  Control flow is SALU only (wave-uniform), with long branches
(s_setpc) because bodies exceed s_cbranch's +-128 KiB reach.

Output: a list of instruction tuples (mnemonic, operands...) where
operands are ints (VGPR n: n, AGPR n: 256+n, SGPR n: 512+n), ("k", value)
for constants, or label strings; see render.py / sim.py.
"""
import os

import gen_fl
from dsl import Loop, If, Op, SUBC, NL, MASK, QL, QINV28, KQ, Q, BINV_OUTER, BINV_PAD, BINV_C

A_BASE, S_BASE = 256, 512
VCC = S_BASE + 106


def V(n): return n
def A(n): return A_BASE + n
def S(n): return S_BASE + n
def K(x): return ("k", x)


ACC = 0
M0 = 2
LOFF, ORACC = 16, 17               # tid * 8 (LDS / spill lane offset); spare
GID, ADDR = 14, 12                 # work-area temporaries of the record I/O code
VSLOT0, NV = 18, 17
NA = 18
NL_SLOTS = 11
SLOT_BYTES = NL * 4 * 64          # 3584: one Fq for 64 lanes
SQ, SQINV, SKQ = 80, 94, 95
# SGPR map
S_KARG = 0          # s[0:1] kernarg pointer
S_WG = 2            # workgroup id
S_ARG = 4           # s[4:13] five 8-byte kernel args
S_WS = 14           # s[14:15] this wave's workspace base
S_TMP = 16          # s[16:17] address temporary
S_EXEC = 18         # s[18:19] saved exec
S_CNT = 20          # s20.. loop counters by depth
S_MASK = 24         # s[24+2d : 25+2d] branch masks by depth
S_JMP = 30          # s[30:31] long-branch temporary
S_VALID = 36        # s[36:37] lane mask: output valid (not infinity / f != 0)
S_LINE = 96         # s[96:97] current line of a shared line table (MillerLoopSharedCfg)
ZERO = 17           # v17 = 0 in kernels with a line table (the wave-uniform load offset)
LINE_BYTES = 6 * NL * 4   # one line: six 14-limb values, 336 B


class AllocError(Exception):
    pass


class ValState:
    __slots__ = ("val", "locs", "uses", "var")

    def __init__(self, val):
        self.val = val
        self.locs = set()   # ("V"|"A"|"L"|"M", k)
        self.uses = []      # item positions (in the defining block) that read it
        self.var = None     # name of the variable whose home holds it (getvar values)


S_ODD = 40          # s[40:41] lane mask of the odd lanes (lane pairs: role 1)
# s[42:80) subtraction constants (loaded by the prologue): the SUBC[1] and
# SUBC[2] limb tables, then (two SGPRs each: limb 0..12, limb 13) the wide
# subtraction constants whose limbs 0..12 are equal; a - b = a + C - b is then
# one v_sad_u32 per limb (|C_i - b_i| + a_i, C_i >= b_i by the bound tracking)
S_CTAB, S_CTAB_END = 42, 80
CTAB_FULL = (1, 2)

# storage configurations: (V slots, A slots, L slots)
STORAGE = {1: (17, 18, int(os.environ.get("PGEN_NL", 11))),  # one wave per SIMD: 256 VGPR + 256 AGPR, 40 KB LDS
           2: (17, 0, 5)}       # two waves per SIMD: 256 VGPR, no AGPR, 20 KB LDS
# PGEN_TWO_WAVES=1 (A/B experiment): one lane per pairing in the two-waves-per-SIMD
# budget of the lane-pair kernels (no AGPRs, 5 LDS slots; render.py declares 256 registers)
TWO_WAVES = os.environ.get("PGEN_TWO_WAVES", "0") == "1"
if TWO_WAVES:
    STORAGE[1] = STORAGE[2]


def plan_ctab(hist):
    """the SGPR constant tables for a program, from a first emission's counts,
    by instructions saved per SGPR: a full table costs 14 SGPRs; a wide constant
    with equal limbs 0..12 costs one SGPR for its top limb plus one per distinct
    repeated limb value"""
    def uni(k, c):
        return k[0] == "csub" and all(x == c[0] for x in c[:NL - 1])
    items = sorted(hist.items(), key=lambda kv: -kv[1] * (7 if uni(*kv[0]) else 1))
    return [kc for kc, n in items if n >= 1]


class Emitter:
    def __init__(self, prog, cfg, ctab_plan=None):
        self.prog = prog
        self.cfg = cfg          # kernel config (kernels.py): loads / stores / flags
        self.code = []
        self.nlabel = 0
        self.NV, self.NA, self.NL = STORAGE[prog.lanes]
        if getattr(cfg, "nl", None) is not None:
            self.NL = cfg.nl
        self.vslot = [None] * self.NV       # ValState or None
        self.aslot = [None] * self.NA       # owner: ("val", vs) | ("var", name) | None
        self.lslot = [None] * self.NL
        self.mslot = []
        self.home = {}                      # var name -> loc
        self.states = {}                    # val id -> ValState
        self.depth = 0
        self.pinned = set()                 # V slots that must not be evicted now
        self.stats = {}
        self.recent_vwrite = {}             # VGPR -> instruction index of last VALU write
        self.recent_awrite = {}
        self.mem_stores_pending = False    # workspace stores whose completion is not tracked
        self.mstore = {}                    # M slot -> vm count right after its last (tracked) store
        self.debug = False
        self.weight = 1
        self.ensuring = None
        self.pending = {}            # V slot -> ("L" | "M", issue count after its last load)
        self.split_pending = {}      # V slot -> True: raw record words, split when they land
        self.vm_issued = 0
        self.lgkm_issued = 0
        self.items = None            # the block being allocated (prefetch lookahead)
        self.defer_vm_wait = False   # batch the waits of one operation's HBM reloads
        self.vm_wait_owed = False
        self.vm_owed_seq = 0
        self.ctab = {}               # constant key -> ("full", sgpr base) | ("uni", sgpr of limbs 0..12)
        self.ctab_init = []          # (sgpr, value) loaded by the prologue
        self.sub_hist = {}           # (constant key, limbs) -> dynamic count (plan_ctab)
        self.ctab_next = S_CTAB
        self.ctab_fixed = False
        if os.environ.get("PGEN_SAD", "1") == "1":
            shared = {}          # repeated limb value -> its SGPR
            for key, c in (ctab_plan if ctab_plan is not None else [(("sub", ub), SUBC[ub]) for ub in CTAB_FULL]):
                if key[0] == "csub" and all(x == c[0] for x in c[:NL - 1]):
                    need = 1 + (c[0] not in shared)
                    if self.ctab_next + need > S_CTAB_END:
                        continue
                    if c[0] not in shared:
                        shared[c[0]] = self.ctab_next
                        self.ctab_init.append((self.ctab_next, c[0]))
                        self.ctab_next += 1
                    self.ctab[key] = ("uni", shared[c[0]], self.ctab_next)
                    self.ctab_init.append((self.ctab_next, c[NL - 1]))
                    self.ctab_next += 1
                    continue
                if self.ctab_next + NL > S_CTAB_END:
                    continue
                self.ctab[key] = ("full", self.ctab_next)
                self.ctab_init += [(self.ctab_next + i, v) for i, v in enumerate(c)]
                self.ctab_next += NL
            self.ctab_fixed = ctab_plan is not None

    # ---------------- emission helpers ----------------
    VMEM = ("global_load_dwordx2", "global_load_dword", "global_store_dwordx2", "global_store_byte",
            "global_store_dwordx2_s", "global_load_dwordx2_s", "global_load_lds_dwordx4")

    def i(self, *t):
        self.code.append(t)
        self.dyn_instr = getattr(self, "dyn_instr", 0) + self.weight   # loop-weighted estimate
        m = t[0]
        if m in self.VMEM:
            self.vm_issued += 1
        elif m.startswith("ds_"):
            self.lgkm_issued += 1
        elif m == "s_waitcnt_vm0":
            self.retire_pending(lambda v: v[0] == "M")
            self.mstore = {}
            self.mem_stores_pending = False
        elif m == "s_waitcnt_lgkm0":
            self.retire_pending(lambda v: v[0] == "L")

    def label(self):
        self.nlabel += 1
        return ".L%s_%d" % (self.prog.name, self.nlabel)

    def bump(self, k, n=1):
        self.stats[k] = self.stats.get(k, 0) + n
        # dynamic estimate: weighted by the trip counts of the enclosing loops
        self.stats["dyn_" + k] = self.stats.get("dyn_" + k, 0) + n * self.weight

    @staticmethod
    def vbase(k):
        return VSLOT0 + 14 * k

    # ---------------- slot bookkeeping ----------------
    def free_vslot(self):
        for k in range(self.NV):
            if self.vslot[k] is None and k not in self.pinned:
                return k
        return None

    def next_use(self, vs, pos):
        for u in vs.uses:
            if u > pos:
                return u
        return 1 << 30

    def retire_pending(self, done):
        """drop the pending entries done(entry) says have landed; a raw record
        value (split_pending: a per-lane tload) is split into its limbs now"""
        gone = [k for k, v in self.pending.items() if done(v)]
        for k in gone:
            del self.pending[k]
        for k in gone:
            if self.split_pending.pop(k, False):
                self.cfg.emit_split(self, self.vbase(k))

    def wait_pending(self, slots=None):
        """complete the in-flight prefetches of the given V slots (default all),
        with counters that leave younger memory operations outstanding"""
        slots = list(self.pending) if slots is None else [k for k in slots if k in self.pending]
        need = {"L": None, "M": None}
        for k in slots:
            kind, seq = self.pending[k]
            need[kind] = seq if need[kind] is None else max(need[kind], seq)
        if need["L"] is not None:
            n = min(15, self.lgkm_issued - need["L"])
            self.i("s_waitcnt_lgkm", n)
            done = self.lgkm_issued - n
            self.retire_pending(lambda v: v[0] == "L" and v[1] <= done)
        if need["M"] is not None:
            n = min(63, self.vm_issued - need["M"])
            self.i("s_waitcnt_vm", n)
            done = self.vm_issued - n
            self.retire_pending(lambda v: v[0] == "M" and v[1] <= done)

    def wait_vm_count(self, n):
        """s_waitcnt vmcnt(n); retire the tracked stores / prefetches it completes"""
        self.i("s_waitcnt_vm", n)
        done = self.vm_issued - n
        self.mstore = {k: q for k, q in self.mstore.items() if q > done}
        self.retire_pending(lambda v: v[0] == "M" and v[1] <= done)

    def untrack_stores(self):
        """control-flow merge / loop back edge: the static issue counts no longer
        describe what is in flight, so the next workspace load waits for all"""
        self.mem_stores_pending = True
        self.mstore = {}

    def get_vslot(self, pos, avoid=()):
        k = self.free_vslot()
        if k is not None:
            if k in self.pending:
                self.wait_pending([k])
            return k
        # Belady, cost-weighted: a value with a copy elsewhere is dropped for
        # free, so it is preferred unless it is needed much sooner
        best, bk = -1, None
        for k in range(self.NV):
            if k in avoid or k in self.pinned:
                continue
            vs = self.vslot[k]
            nu = self.next_use(vs, pos) - pos
            score = nu * self.drop_weight(vs)
            if score > best:
                best, bk = score, k
        if bk is None:
            raise AllocError("no evictable V slot")
        if bk in self.pending:   # a late load must not land over the new value
            self.wait_pending([bk])
        self.evict(bk, pos)
        return bk

    # Belady weights: dropping a value with a copy in an AGPR costs 14 moves to
    # reload, in LDS 7 loads, in the HBM workspace 7 loads + latency + traffic;
    # a value without a copy costs a spill first (PGEN_DROP_W: A/B experiments)
    DROP_W = tuple(float(x) for x in os.environ.get("PGEN_DROP_W", "3,3,3,1").split(","))

    def drop_weight(self, vs):
        kinds = {l[0] for l in vs.locs if l[0] != "V"}
        if not kinds:
            return self.DROP_W[3]
        return max(self.DROP_W["ALM".index(k)] for k in kinds)

    # a value whose only other copy is in the HBM workspace and that is read
    # again within KEEP_M operations is copied to a free AGPR / LDS slot as it
    # leaves its V slot, so its next uses reload on chip (PGEN_KEEP_M=0: off)
    KEEP_M = int(os.environ.get("PGEN_KEEP_M", "0"))

    def free_onchip(self):
        for kind, tab in (("A", self.aslot), ("L", self.lslot)):
            for j, o in enumerate(tab):
                if o is None:
                    return (kind, j)
        return None

    def evict(self, k, pos):
        vs = self.vslot[k]
        vs.locs.discard(("V", k))
        if (self.KEEP_M and vs.locs and all(l[0] == "M" for l in vs.locs)
                and self.next_use(vs, pos) - pos <= self.KEEP_M and vs.val.id in self.local_ids):
            loc = self.free_onchip()
            if loc is not None:
                self.copy(("V", k), loc)
                self.own(loc, vs)
                vs.locs.add(loc)
                self.bump("keep_" + loc[0])
        if not vs.locs:
            loc = self.tier_slot(vs, pos)
            self.copy(("V", k), loc)
            self.own(loc, vs)
            vs.locs.add(loc)
            self.bump("spill_" + loc[0])
        self.vslot[k] = None

    def tier_slot(self, vs, pos):
        """spill destination: a free A or L slot; else demote the A/L-resident
        spill with the furthest next use to M if it is needed later than vs"""
        for kind, tab in (("A", self.aslot), ("L", self.lslot)):
            for k, o in enumerate(tab):
                if o is None:
                    return (kind, k)
        mine = self.next_use(vs, pos)
        best, bl = mine, None
        for kind, tab in (("A", self.aslot), ("L", self.lslot)):
            for k, o in enumerate(tab):
                if (o is not None and o[0] == "val" and o[1].val.id in self.local_ids
                        and o[1] is not self.ensuring and not any(l[0] == "V" and l[1] in self.pinned
                                                                  for l in o[1].locs)):
                    nu = self.next_use(o[1], pos)
                    if nu > best:
                        best, bl = nu, (kind, k)
        if bl is None:
            return self.spill_slot(prefer="M")
        other = (self.aslot if bl[0] == "A" else self.lslot)[bl[1]][1]
        m = self.spill_slot(prefer="M")
        self.copy_via_work(bl, m)
        other.locs.discard(bl)
        other.locs.add(m)
        self.own(m, other)
        self.bump("demote_" + bl[0])
        return bl

    def copy_via_work(self, src, dst):
        """A/L -> M through the work area v0..v13 (free between operations)"""
        sk, s = src
        if sk == "A":
            for j in range(14):
                self.i("v_accvgpr_read_b32", j, A(14 * s + j))
        else:
            for j in range(7):
                self.i("ds_read_b64", 2 * j, LOFF, s * SLOT_BYTES + 512 * j)
            self.i("s_waitcnt_lgkm0")
        d = dst[1]
        self.i("s_add_u32", S(S_TMP), S(S_WS), K(d * SLOT_BYTES))
        self.i("s_addc_u32", S(S_TMP + 1), S(S_WS + 1), K(0))
        for j in range(7):
            self.i("global_store_dwordx2_s", LOFF, 2 * j, S(S_TMP), 512 * j)
        self.mstore[d] = self.vm_issued

    def own(self, loc, vs):
        kind, k = loc
        if kind == "A":
            self.aslot[k] = ("val", vs)
        elif kind == "L":
            self.lslot[k] = ("val", vs)
        elif kind == "M":
            self.mslot[k] = ("val", vs)
        elif kind == "V":
            self.vslot[k] = vs

    def spill_slot(self, prefer="A"):
        order = {"A": "ALM", "L": "LAM", "M": "MLA"}[prefer]
        for kind in order:
            tab = {"A": self.aslot, "L": self.lslot, "M": self.mslot}[kind]
            for k, o in enumerate(tab):
                if o is None:
                    return (kind, k)
            if kind == "M":
                self.mslot.append(None)
                return ("M", len(self.mslot) - 1)
        raise AllocError("no spill slot")

    def release_loc(self, loc, vs):
        kind, k = loc
        tab = {"A": self.aslot, "L": self.lslot, "M": self.mslot}.get(kind)
        if kind == "V":
            if self.vslot[k] is vs:
                self.vslot[k] = None
        elif tab[k] == ("val", vs):
            tab[k] = None

    def kill(self, vs):
        for loc in list(vs.locs):
            self.release_loc(loc, vs)
        vs.locs.clear()

    # ---------------- data movement ----------------
    def copy(self, src, dst, wait=True):
        """move one Fq between locations (src and dst kinds may differ);
        wait=False leaves an L/M -> V load in flight (prefetch)"""
        sk, s = src
        dk, d = dst
        self.bump("move_%s%s" % (sk, dk))
        if sk == "V" and dk == "V":
            for j in range(7):
                self.i("v_mov_b64", self.vbase(d) + 2 * j, self.vbase(s) + 2 * j)
        elif sk == "V" and dk == "A":
            for j in range(14):
                self.i("v_accvgpr_write_b32", A(14 * d + j), self.vbase(s) + j)
        elif sk == "A" and dk == "V":
            for j in range(14):
                self.i("v_accvgpr_read_b32", self.vbase(d) + j, A(14 * s + j))
        elif sk == "V" and dk == "L":
            for j in range(7):
                self.i("ds_write_b64", LOFF, self.vbase(s) + 2 * j, d * SLOT_BYTES + 512 * j)
        elif sk == "L" and dk == "V":
            for j in range(7):
                self.i("ds_read_b64", self.vbase(d) + 2 * j, LOFF, s * SLOT_BYTES + 512 * j)
            if wait:
                self.i("s_waitcnt_lgkm0")
        elif sk == "V" and dk == "M":
            self.i("s_add_u32", S(S_TMP), S(S_WS), K(d * SLOT_BYTES))
            self.i("s_addc_u32", S(S_TMP + 1), S(S_WS + 1), K(0))
            for j in range(7):
                self.i("global_store_dwordx2_s", LOFF, self.vbase(s) + 2 * j, S(S_TMP), 512 * j)
            self.mstore[d] = self.vm_issued
        elif sk == "M" and dk == "V":
            if self.mem_stores_pending:
                self.i("s_waitcnt_vm0")
            elif s in self.mstore:
                # vector memory operations complete in issue order: wait only
                # until this slot's store is done
                self.wait_vm_count(min(63, self.vm_issued - self.mstore[s]))
            self.i("s_add_u32", S(S_TMP), S(S_WS), K(s * SLOT_BYTES))
            self.i("s_addc_u32", S(S_TMP + 1), S(S_WS + 1), K(0))
            for j in range(7):
                self.i("global_load_dwordx2_s", self.vbase(d) + 2 * j, LOFF, S(S_TMP), 512 * j)
            if not wait:
                pass
            elif self.defer_vm_wait:
                self.vm_wait_owed = True
                self.vm_owed_seq = self.vm_issued
            else:
                self.i("s_waitcnt_vm0")
        else:
            # via a V slot is the caller's job
            raise AllocError("copy %s -> %s" % (src, dst))

    def best_src(self, vs):
        for kind in "VALM":
            for loc in vs.locs:
                if loc[0] == kind:
                    return loc
        raise AllocError("value %r has no location" % vs.val)

    def ensure_v(self, vs, pos, avoid):
        for loc in vs.locs:
            if loc[0] == "V":
                return loc[1]
        self.ensuring = vs
        k = self.get_vslot(pos, avoid)   # may demote other spills (not vs)
        self.ensuring = None
        src = self.best_src(vs)
        self.copy(src, ("V", k))
        self.vslot[k] = vs
        vs.locs.add(("V", k))
        self.bump("reload_" + src[0])
        return k

    # ---------------- ops ----------------
    def emit_sop(self, pairs, d, signed=False):
        """signed (dsl.Prog._ssop, one pair, b's limbs signed): the products by
        v_mad_i64_i32 into a signed accumulator, arithmetic shifts between
        columns, and the last Montgomery digit + 2^28 (the result + q, so it
        stays positive); the reduction's products are unsigned either way"""
        first = True
        acc = (ACC, ACC + 1)
        mad = "v_mad_i64_i32" if signed else "v_mad_u64_u32"
        for k in range(2 * NL - 1):
            for a, b in pairs:
                for i in range(max(0, k - NL + 1), min(k, NL - 1) + 1):
                    self.i(mad, ACC, a + i, b + k - i, K(0) if first else ACC)
                    first = False
            for i in range(max(0, k - NL + 1), min(k - 1, NL - 1) + 1):
                self.i("v_mad_u64_u32", ACC, M0 + i, S(SQ + k - i), ACC)
            if k < NL:
                self.i("v_mul_lo_u32", M0 + k, ACC, S(SQINV))
                self.i("v_and_b32", M0 + k, K(MASK), M0 + k)
                if signed and k == NL - 1:
                    self.i("v_or_b32", M0 + k, K(1 << 28), M0 + k)
                self.i("v_mad_u64_u32", ACC, M0 + k, S(SQ), ACC)
            else:
                self.i("v_and_b32", d + k - NL, K(MASK), ACC)
            self.i("v_ashrrev_i64" if signed else "v_lshrrev_b64", ACC, K(28), ACC)
        self.i("v_mov_b32", d + NL - 1, ACC)
        del acc

    def emit_pdiff(self, a, d):
        """d = (a0 - a1 | a0), signed limbs: w = VCC ? 0 : partner's a (v15 = 0,
        VCC = the odd lanes), then d = a of lane 0 (DPP broadcast) - w.  w lives in
        d; the cndmasks alternate with the subs (back-to-back VOP2 cndmasks issue
        slowly).  d must not alias a."""
        self.i("s_mov_b64", VCC, S(S_ODD))
        self.i("v_mov_b32", 15, K(0))
        self.i("s_nop", 1)   # VALU write -> DPP read of the same VGPR: 2 wait states
        for i in range(NL):
            self.i("v_cndmask_b32_dpp_swap", d + i, a + i, 15)
            if i:
                self.i("v_sub_u32_dpp_bcast0", d + i - 1, a + i - 1, d + i - 1)
        self.i("v_sub_u32_dpp_bcast0", d + NL - 1, a + NL - 1, d + NL - 1)

    def emit_red(self, x, d):
        self.i("v_mad_u64_u32", ACC, x + 12, S(SKQ), K(0))
        self.i("v_mad_u64_u32", 4, x + 13, S(SKQ), K(0))
        self.i("v_lshrrev_b64", ACC, K(28), ACC)
        self.i("v_lshl_add_u64", ACC, 4, K(0), ACC)
        self.i("v_lshrrev_b32", 2, K(4), ACC + 1)          # k
        self.i("v_sub_u32", 3, K(0), 2)                     # -k
        for i in range(NL):
            self.i("v_mad_u64_u32", ACC, x + i, K(1), K(0) if i == 0 else ACC)
            self.i("v_mad_i64_i32", ACC, 3, S(SQ + i), ACC)
            if i < NL - 1:
                self.i("v_and_b32", d + i, K(MASK), ACC)
                self.i("v_ashrrev_i64", ACC, K(28), ACC)
            else:
                self.i("v_mov_b32", d + i, ACC)

    def emit_norm(self, x, d):
        """carry pass: limbs 0..12 below 2^28, value unchanged (dsl.norm_limbs);
        carry in v1, running sum in v0 (x may equal d: each limb is read first)"""
        self.i("v_lshrrev_b32", ACC + 1, K(28), x)
        self.i("v_and_b32", d, K(MASK), x)
        for i in range(1, NL - 1):
            self.i("v_add_u32", ACC, x + i, ACC + 1)
            self.i("v_and_b32", d + i, K(MASK), ACC)
            self.i("v_lshrrev_b32", ACC + 1, K(28), ACC)
        self.i("v_add_u32", d + NL - 1, x + NL - 1, ACC + 1)

    def emit_add(self, a, b, d):
        for i in range(NL):
            self.i("v_add_u32", d + i, a + i, b + i)

    def ctab_reg(self, key, c):
        """SGPR of limb i of constant c (or None): the tables planned by plan_ctab
        (or full SUBC[1], SUBC[2] tables, then constants with equal limbs 0..12,
        two SGPRs each, while the area lasts)"""
        hk = (key, tuple(c))
        self.sub_hist[hk] = self.sub_hist.get(hk, 0) + self.weight
        if os.environ.get("PGEN_SAD", "1") != "1":
            return None
        e = self.ctab.get(key)
        if (e is None and not self.ctab_fixed and all(x == c[0] for x in c[:NL - 1])
                and self.ctab_next + 2 <= S_CTAB_END):
            e = self.ctab[key] = ("uni", self.ctab_next, self.ctab_next + 1)
            self.ctab_init += [(self.ctab_next, c[0]), (self.ctab_next + 1, c[NL - 1])]
            self.ctab_next += 2
        if e is None:
            return None
        if e[0] == "full":
            return lambda i: S(e[1] + i)
        return lambda i: S(e[1] if i < NL - 1 else e[2])

    def emit_sub(self, a, b, d, ub):
        c = SUBC[ub]
        r = self.ctab_reg(("sub", ub), tuple(c))
        if r is not None:
            for i in range(NL):
                self.i("v_sad_u32", d + i, r(i), b + i, a + i)
            return
        if d == b:
            assert a != b
            for i in range(NL):
                self.i("v_sub_u32", d + i, K(c[i]), b + i)
                self.i("v_add_u32", d + i, a + i, d + i)
        else:
            for i in range(NL):
                self.i("v_add_u32", d + i, K(c[i]), a + i)
                self.i("v_sub_u32", d + i, d + i, b + i)

    def emit_csub(self, a, b, d, c):
        """a + C - b limb-wise, C given (wide-value halves)"""
        r = self.ctab_reg(("csub", tuple(c)), c)
        if r is not None:
            for i in range(NL):
                self.i("v_sad_u32", d + i, r(i), b + i, a + i)
            return
        if d == b:
            assert a != b
            for i in range(NL):
                self.i("v_sub_u32", d + i, K(c[i]), b + i)
                self.i("v_add_u32", d + i, a + i, d + i)
        else:
            for i in range(NL):
                self.i("v_add_u32", d + i, K(c[i]), a + i)
                self.i("v_sub_u32", d + i, d + i, b + i)

    def emit_wsop(self, pairs, dlo, dhi):
        """sum a*b as 28 normalized limbs, no reduction: column k -> limb k"""
        first = True
        for k in range(2 * NL - 1):
            for a, b in pairs:
                for i in range(max(0, k - NL + 1), min(k, NL - 1) + 1):
                    self.i("v_mad_u64_u32", ACC, a + i, b + k - i, K(0) if first else ACC)
                    first = False
            self.i("v_and_b32", (dlo + k) if k < NL else (dhi + k - NL), K(MASK), ACC)
            self.i("v_lshrrev_b64", ACC, K(28), ACC)
        self.i("v_mov_b32", dhi + NL - 1, ACC)

    def emit_wnorm(self, lo, hi, dlo, dhi):
        """carry propagation over the 28 limbs (carry in v0, sum in v1)"""
        for k in range(2 * NL):
            src = (lo + k) if k < NL else (hi + k - NL)
            dst = (dlo + k) if k < NL else (dhi + k - NL)
            if k == 0:
                self.i("v_lshrrev_b32", ACC, K(28), src)
                self.i("v_and_b32", dst, K(MASK), src)
            elif k < 2 * NL - 1:
                self.i("v_add_u32", ACC + 1, src, ACC)
                self.i("v_lshrrev_b32", ACC, K(28), ACC + 1)
                self.i("v_and_b32", dst, K(MASK), ACC + 1)
            else:
                self.i("v_add_u32", dst, src, ACC)

    def emit_wred(self, lo, hi, d):
        """Montgomery reduction of lo + hi 2^392: the reduction half of a sop
        with the column inputs taken from the wide value"""
        for k in range(2 * NL - 1):
            src = (lo + k) if k < NL else (hi + k - NL)
            if k == 0:
                self.i("v_mov_b32", ACC, src)
                self.i("v_mov_b32", ACC + 1, K(0))
            else:
                self.i("v_mad_u64_u32", ACC, src, K(1), ACC)
            for i in range(max(0, k - NL + 1), min(k - 1, NL - 1) + 1):
                self.i("v_mad_u64_u32", ACC, M0 + i, S(SQ + k - i), ACC)
            if k < NL:
                self.i("v_mul_lo_u32", M0 + k, ACC, S(SQINV))
                self.i("v_and_b32", M0 + k, K(MASK), M0 + k)
                self.i("v_mad_u64_u32", ACC, M0 + k, S(SQ), ACC)
            else:
                self.i("v_and_b32", d + k - NL, K(MASK), ACC)
            self.i("v_lshrrev_b64", ACC, K(28), ACC)
        self.i("v_add_u32", d + NL - 1, hi + NL - 1, ACC)

    def emit_neg(self, b, d, ub):
        c = SUBC[ub]
        for i in range(NL):
            self.i("v_sub_u32", d + i, K(c[i]), b + i)

    def emit_swap(self, a, d):
        self.i("s_nop", 1)   # VALU write -> DPP read of the same VGPR: 2 wait states
        for i in range(NL):
            self.i("v_mov_b32_dpp_swap", d + i, a + i)

    def emit_dppadd(self, a, b, d, perm):
        self.i("s_nop", 1)   # VALU write -> DPP read of the same VGPR: 2 wait states
        for i in range(NL):
            self.i("v_add_u32_dpp", d + i, a + i, b + i, perm)

    def emit_bcast(self, a, d, r):
        self.i("s_nop", 1)   # VALU write -> DPP read of the same VGPR: 2 wait states
        for i in range(NL):
            self.i("v_mov_b32_dpp_bcast", d + i, a + i, r)

    def emit_pairz(self, a, d, key):
        """d = C - a (every lane), then d = VCC ? a : d of the partner lane
        (v_cndmask_b32_dpp, VCC = the odd lanes): lane 0 gets C - a1, lane 1
        its a.  The cndmask of limb i comes three instructions after the sub
        that writes limb i (a DPP read needs two wait states after the VALU
        write) and the cndmasks alternate with the subs (back-to-back VOP2
        cndmasks reading VCC issue at ~19 clk on a lone wave,
        profiles/r03_issue_probe.txt).  d must not alias a."""
        c = SUBC[key]
        self.i("s_mov_b64", VCC, S(S_ODD))
        seq = [("s", 0), ("s", 1), ("s", 2)]
        for i in range(NL):
            seq.append(("c", i))
            if i + 3 < NL:
                seq.append(("s", i + 3))
        at = {}
        for n, (kind, i) in enumerate(seq):
            if kind == "s":
                self.i("v_sub_u32", d + i, K(c[i]), a + i)
                at[i] = n
            else:
                assert n - at[i] - 1 >= 2
                self.i("v_cndmask_b32_dpp_swap", d + i, d + i, a + i)

    def emit_sel(self, a, b, d):
        for i in range(NL):
            self.i("v_cndmask_b32_e64", d + i, a + i, b + i, S(S_ODD))

    def emit_const(self, limbs, d):
        for i in range(NL):
            self.i("v_mov_b32", d + i, K(limbs[i]))

    # ---- zero-test select (dsl.Prog.selz) ----
    def emit_selz(self, tests, a, b, d):
        """d = a where every test (limbs < 2^28, value < 2q) is 0 or q, else b.
        Masks: s[32:33] / s[34:35] / s[38:39] (free outside record I/O and
        binv), the final one in VCC by SALU; a VALU read of an SGPR a VALU
        wrote needs two wait states on gfx950 (only SALU reads follow the
        compares here)."""
        pairs = ((S(32), S(34)), (S(38), S(34)))
        for n, t in enumerate(tests):
            self.i("v_or3_b32", 0, t, t + 1, t + 2)
            for i in range(3, NL, 2):
                if i + 1 < NL:
                    self.i("v_or3_b32", 0, 0, t + i, t + i + 1)
                else:
                    self.i("v_or_b32", 0, 0, t + i)
            for i in range(NL):
                self.i("v_xor_b32", 2 + i, S(SQ + i), t + i)
            self.i("v_or3_b32", 1, 2, 3, 4)
            for i in range(5, 2 + NL, 2):
                if i + 1 < 2 + NL:
                    self.i("v_or3_b32", 1, 1, i, i + 1)
                else:
                    self.i("v_or_b32", 1, 1, i)
            za, zq = pairs[n]
            self.i("v_cmp_eq_u32_e64", za, K(0), 0)
            self.i("v_cmp_eq_u32_e64", zq, K(0), 1)
            self.i("s_or_b64", za, za, zq)
        if len(tests) == 1:
            self.i("s_mov_b64", VCC, S(32))
        else:
            self.i("s_and_b64", VCC, S(32), S(38))
        # the e64 form: back-to-back VOP2 v_cndmask_b32 (implicit VCC) issue at
        # 19 clk on a lone wave, the e64 form at 6 (profiles/r03_issue_probe.txt)
        for i in range(NL):
            self.i("v_cndmask_b32_e64", d + i, b + i, a + i, VCC)

    # ---- in-kernel binary GCD inversion (dsl.Prog.binv, dsl.binv_limbs) ----
    def emit_binv(self, x, d, scratch):
        """d = x^-1 (Fl domain, 0 -> 0) by T. Pornin's optimized binary GCD
        (eprint 2020/972, Algorithm 2) on 28-bit limbs -- the same algorithm as
        pairing_amd/csrc/bgcd.h with k - 1 = 28 so that the exact update's
        division by 2^28 drops one limb.  Exact semantics: dsl.binv_limbs.

        Registers: a, b, u, w = four scratch V slots; work area v0..v15
        (v16 = the lane offset, v17 are kept); s[32:33] s[34:35] s[38:39] VCC
        masks; the outer loop counter at S_CNT + depth.  Every VALU read of an
        SGPR a VALU wrote comes at least two instructions after the write."""
        a, b, u, w = (self.vbase(k) for k in scratch)
        MK = K(MASK)
        # y = x mod q, canonical, into a
        self.emit_red(x, a)
        for li in range(NL):
            self.i("v_subrev_u32", li, K(QL[li]), a + li)
            if li:
                self.i("v_add_u32", li, li, 14)
            self.i("v_ashrrev_i32", 14, K(28), li)
            self.i("v_and_b32", li, MK, li)
        for li in range(NL):
            self.i("v_bfi_b32", a + li, 14, a + li, li)     # a < q ? a : a - q
        for i in range(NL):
            self.i("v_mov_b32", b + i, S(SQ + i))
            self.i("v_mov_b32", u + i, K(1 if i == 0 else 0))
            self.i("v_mov_b32", w + i, K(0))
        cnt = S(S_CNT + self.depth)
        top = self.label()
        self.i("s_mov_b32", cnt, K(BINV_OUTER - 1))
        self.i("label", top)
        w0 = self.weight
        self.weight = w0 * BINV_OUTER
        # -- n = max(len(a | b), 58): top nonzero limb (index v13, value v12),
        #    limbs 2..13 (below limb 2 the max with 58 decides anyway)
        masks = (S(32), S(34), S(38))
        self.i("v_mov_b32", 12, K(1))
        self.i("v_mov_b32", 13, K(1))
        for i in range(2, NL):
            self.i("v_or_b32", i - 2, a + i, b + i)
        # compares rotate over three SGPR pairs so each select is >= 2 wait states after its compare
        order = list(range(2, NL))
        for n, i in enumerate(order):
            self.i("v_cmp_eq_u32_e64", masks[n % 3], K(0), i - 2)
            if n >= 2:
                j = order[n - 2]
                m = masks[(n - 2) % 3]
                self.i("v_cndmask_b32_e64", 12, j - 2, 12, m)      # zero ? old : limb
                self.i("v_cndmask_b32_e64", 13, K(j), 13, m)       # zero ? old : index
        for n in (len(order) - 2, len(order) - 1):
            j = order[n]
            m = masks[n % 3]
            self.i("v_cndmask_b32_e64", 12, j - 2, 12, m)
            self.i("v_cndmask_b32_e64", 13, K(j), 13, m)
        self.i("v_ffbh_u32", 14, 12)
        self.i("v_sub_u32", 15, K(32), 14)
        self.i("v_mad_u32_u24", 15, 13, K(28), 15)           # n = 28 idx + bitlen(limb)
        self.i("v_max_u32", 15, K(58), 15)
        self.i("v_subrev_u32", 15, K(30), 15)                # p = n - 30 >= 28
        self.i("v_mul_u32_u24", 14, K(9363), 15)
        self.i("v_lshrrev_b32", 14, K(18), 14)               # j = p / 28 (exact for p < 392)
        self.i("v_mul_u32_u24", 13, K(28), 14)
        self.i("v_sub_u32", 15, 15, 13)                      # s = p - 28 j
        # -- barrel masks of j: s[32:33] bit 8, s[34:35] bit 4, s[38:39] bit 2, VCC bit 1
        bm = (S(32), S(34), S(38), VCC)
        for bit, m in zip((8, 4, 2, 1), bm):
            self.i("v_and_b32", 12, K(bit), 14)
            if m == VCC:
                self.i("v_cmp_ne_u32", K(0), 12)
            else:
                self.i("v_cmp_ne_u32_e64", m, K(0), 12)
        # -- approximations: xa = v[10:11], xb = v[12:13]
        for src, dst in ((a, 10), (b, 12)):
            for i in range(10):
                self.i("v_cndmask_b32_e64", i, src + i, (src + i + 8) if i + 8 < NL else K(0), bm[0])
            for st, m, cntn in ((4, bm[1], 6), (2, bm[2], 4), (1, bm[3], 3)):
                for i in range(cntn):
                    self.i("v_cndmask_b32_e64", i, i, i + st, m)
            self.i("v_lshl_or_b32", 4, 1, K(28), 0)
            self.i("v_lshrrev_b32", 5, K(4), 1)
            self.i("v_lshl_or_b32", 5, 2, K(24), 5)
            self.i("v_lshrrev_b64", 4, 15, 4)
            self.i("v_and_b32", 4, K((1 << 30) - 1), 4)
            self.i("v_lshl_or_b32", dst, 4, K(28), src)
            self.i("v_lshrrev_b32", dst + 1, K(4), 4)
        # -- 28 inner steps: f0 v6, g0 v7, f1 v8, g1 v9
        for r, v in ((6, 1), (7, 0), (8, 0), (9, 1)):
            self.i("v_mov_b32", r, K(v))
        for _ in range(28):
            self.i("v_and_b32", 0, K(1), 10)
            self.i("v_cmp_lt_u64_e64", S(38), 10, 12)          # lt
            self.i("v_cmp_ne_u32_e64", S(34), K(0), 0)          # odd
            self.i("s_and_b64", VCC, S(34), S(38))              # swap = odd & lt
            self.i("v_cndmask_b32_e64", 0, 10, 12, VCC)  # XA = swap ? xb : xa
            self.i("v_cndmask_b32_e64", 1, 11, 13, VCC)
            self.i("v_cndmask_b32_e64", 12, 12, 10, VCC)  # xb' = swap ? xa : xb
            self.i("v_cndmask_b32_e64", 13, 13, 11, VCC)
            self.i("v_cndmask_b32_e64", 4, 6, 8, VCC)  # FA = swap ? f1 : f0
            self.i("v_cndmask_b32_e64", 8, 8, 6, VCC)  # FB
            self.i("v_cndmask_b32_e64", 5, 7, 9, VCC)  # GA
            self.i("v_cndmask_b32_e64", 9, 9, 7, VCC)  # GB
            self.i("v_sub_co_u32", 2, 0, 12)                    # XA - XB (borrow in VCC)
            self.i("v_sub_u32", 14, 4, 8)
            self.i("v_sub_u32", 15, 5, 9)
            self.i("v_subb_co_u32", 3, 1, 13)
            self.i("v_cndmask_b32_e64", 6, 4, 14, S(34))        # f0' = odd ? FA - FB : FA
            self.i("v_cndmask_b32_e64", 7, 5, 15, S(34))
            self.i("v_lshlrev_b32", 8, K(1), 8)                 # f1' = 2 FB
            self.i("v_lshlrev_b32", 9, K(1), 9)
            self.i("v_cndmask_b32_e64", 10, 0, 2, S(34))        # xa' = (odd ? XA - XB : XA) / 2
            self.i("v_cndmask_b32_e64", 11, 1, 3, S(34))
            self.i("v_lshrrev_b64", 10, K(1), 10)
        # -- (a, b) <- ((a f0 + b g0), (a f1 + b g1)) / 2^28, in place (column i -> limb i - 1)
        self.comb_columns(((a, 6, b, 7, None), (b, 9, a, 8, None)))
        # -- negative results: negate the limbs and the factor row
        for src, mreg in ((a, 10), (b, 11)):
            self.i("v_ashrrev_i32", mreg, K(31), src + NL - 1)
            self.i("v_and_b32", 12, MK, mreg)
            self.i("v_lshrrev_b32", 13, K(31), src + NL - 1)
            for i in range(NL - 1):
                self.i("v_xad_u32", 15, src + i, 12, 13)
                self.i("v_and_b32", src + i, MK, 15)
                self.i("v_lshrrev_b32", 13, K(28), 15)
            self.i("v_xad_u32", src + NL - 1, src + NL - 1, mreg, 13)
        for r, mreg in ((6, 10), (7, 10), (8, 11), (9, 11)):
            self.i("v_xor_b32", r, r, mreg)
            self.i("v_sub_u32", r, r, mreg)
        # -- (u, w) <- ((u f0 + w g0), (u f1 + w g1)) / 2^28 mod q (one Montgomery digit each)
        self.comb_columns(((u, 6, w, 7, 4), (w, 9, u, 8, 5)))
        self.weight = w0
        self.i("s_sub_u32", cnt, cnt, K(1))
        self.i("s_cmp_ge_i32", cnt, K(0))
        self.i("long_cbranch_scc1", top)
        # -- w + 32 q >= 0, normalized; times R'^3 (one Montgomery product)
        pad = gen_fl.limbs(BINV_PAD * Q)
        for i in range(NL):
            self.i("v_add_u32", 1, K(pad[i]), w + i)
            if i == NL - 1:
                self.i("v_add_u32", w + i, 1, 0)
                break
            if i:
                self.i("v_add_u32", 1, 1, 0)
            self.i("v_and_b32", w + i, MK, 1)
            self.i("v_lshrrev_b32", 0, K(28), 1)
        self.emit_const(gen_fl.limbs(BINV_C), a)
        self.emit_sop([(w, a)], d)

    def comb_columns(self, rows):
        """two signed linear combinations of the 14-limb values, divided by
        2^28 in place: for each row (x, fx, y, fy, kreg) the accumulator gets
        x_i f + y_i g (+ k q_i when kreg names the VGPR of the Montgomery digit,
        k = -(column 0) q^-1 mod 2^28); column i's low 28 bits replace limb
        i - 1 of x, the final carry is limb 13 (signed).  Accumulators v[0:1],
        v[2:3]; the rows' x must be the two values being replaced, each row
        reading both before either is written."""
        accs = (0, 2)
        for i in range(NL):
            for (x, fx, y, fy, kreg), acc in zip(rows, accs):
                self.i("v_mad_i64_i32", acc, x + i, fx, K(0) if i == 0 else acc)
                self.i("v_mad_i64_i32", acc, y + i, fy, acc)
                if kreg is not None:
                    if i == 0:
                        self.i("v_mul_lo_u32", kreg, acc, S(SQINV))
                        self.i("v_and_b32", kreg, K(MASK), kreg)
                    self.i("v_mad_i64_i32", acc, kreg, S(SQ + i), acc)
            if i:
                for (x, _, _, _, _), acc in zip(rows, accs):
                    self.i("v_and_b32", x + i - 1, K(MASK), acc)
            for acc in accs:
                self.i("v_ashrrev_i64", acc, K(28), acc)
        for (x, _, _, _, _), acc in zip(rows, accs):
            self.i("v_mov_b32", x + NL - 1, acc)

    # ---------------- blocks ----------------
    def analyse(self, block):
        """ValStates + use positions for the values defined in `block`"""
        for pos, it in enumerate(block.items):
            if isinstance(it, Op):
                for v in it.srcs:
                    self.states[v.id].uses.append(pos)
                if it.dst is not None:
                    self.states[it.dst.id] = ValState(it.dst)
                if it.dst2 is not None:
                    self.states[it.dst2.id] = ValState(it.dst2)

    def var_ranges(self, block):
        """for each var touched in `block` (at any depth): (first, last) item position"""
        rng = {}

        def touch(name, pos):
            f, l = rng.get(name, (pos, pos))
            rng[name] = (min(f, pos), max(l, pos))

        def walk(b, pos):
            for it in b.items:
                if isinstance(it, (Loop, If)):
                    walk(it.body, pos)
                elif it.kind in ("getvar", "setvar"):
                    touch(it.imm, pos)

        for pos, it in enumerate(block.items):
            if isinstance(it, (Loop, If)):
                walk(it.body, pos)
            elif it.kind in ("getvar", "setvar"):
                touch(it.imm, pos)
        return rng

    def alloc_home(self, name, pos):
        var = self.prog.vars[name]
        pref = (var.home or "A")[0] if isinstance(var.home, str) else "A"
        loc = self.spill_slot(prefer=pref)
        if pref != "M" and loc[0] != pref:
            # the preferred tier is full of spills: push the coldest one to M
            tab = self.aslot if pref == "A" else self.lslot
            best, bk = -1, None
            for k, o in enumerate(tab):
                if o is not None and o[0] == "val":
                    nu = self.next_use(o[1], pos)
                    if nu > best:
                        best, bk = nu, k
            if bk is not None:
                other = tab[bk][1]
                m = self.spill_slot(prefer="M")
                self.copy_via_work((pref, bk), m)
                other.locs.discard((pref, bk))
                other.locs.add(m)
                self.own(m, other)
                self.bump("demote_home_" + pref)
                tab[bk] = None
                loc = (pref, bk)
        tab = {"A": self.aslot, "L": self.lslot, "M": self.mslot}[loc[0]]
        tab[loc[1]] = ("var", name)
        self.home[name] = loc

    def free_home(self, name, pos):
        """the variable is dead; values read from it may still be live and keep
        the slot as their own storage"""
        loc = self.home.pop(name)
        tab = {"A": self.aslot, "L": self.lslot, "M": self.mslot}[loc[0]]
        tab[loc[1]] = None
        for vs in self.states.values():
            if loc in vs.locs:
                if self.next_use(vs, pos) == 1 << 30:
                    vs.locs.discard(loc)
                elif tab[loc[1]] is None:
                    tab[loc[1]] = ("val", vs)
                else:
                    vs.locs.discard(loc)
                    if not vs.locs:
                        raise AllocError("two live readers of dead variable %s" % name)

    def run_block(self, block, top=False):
        self.analyse(block)
        saved_ids = getattr(self, "local_ids", set())
        self.local_ids = self.block_vals(block)
        saved_items = self.items
        self.items = block.items
        if top:
            self.index_vars(block)
            vr = self.var_ranges(block)
        else:
            # variables that live only inside this block, written before any
            # read in each pass: their homes exist only over their range here
            loc = self.local_vars.get(id(block), ())
            vr = {n: r for n, r in self.var_ranges(block).items() if n in loc}
        for pos, it in enumerate(block.items):
            for name, (f, _) in vr.items():
                if f == pos and name not in self.home:
                    self.alloc_home(name, pos)
            if isinstance(it, (Loop, If)):
                self.park(block, pos)
                self.run_construct(it)
            else:
                self.run_op(it, pos)
            for name, (_, l) in vr.items():
                if l == pos and name in self.home:
                    self.free_home(name, pos)
        # everything defined here is dead now
        self.wait_pending()
        self.items = saved_items
        for k in range(self.NV):
            vs = self.vslot[k]
            if vs is not None and vs.val.id in self.local_ids:
                self.kill(vs)
        self.local_ids = saved_ids

    def index_vars(self, root):
        """self.local_vars: block id -> the variables whose every access lies in
        that block's subtree and whose first access there is a setvar directly
        in the block (so no value crosses a back edge of an enclosing loop);
        the innermost such block gets the variable (PGEN_LOCAL_HOMES=0: every
        home lives at the top level, round 2)"""
        self.local_vars = {}
        if os.environ.get("PGEN_LOCAL_HOMES", "1") != "1":
            return
        parent, where, first = {}, {}, {}

        def walk(block, par):
            parent[id(block)] = par
            for it in block.items:
                if isinstance(it, (Loop, If)):
                    walk(it.body, id(block))
                elif it.kind in ("getvar", "setvar"):
                    where.setdefault(it.imm, set()).add(id(block))
                    first.setdefault((id(block), it.imm), it.kind)
        walk(root, None)

        def ancestors(b):
            out = []
            while b is not None:
                out.append(b)
                b = parent[b]
            return out

        for name, blocks in where.items():
            common = None
            for b in blocks:
                a = ancestors(b)
                common = a if common is None else [x for x in common if x in a]
            # innermost common ancestor whose own first access is a setvar and
            # that holds the first access of the subtree
            for b in common:
                if b == id(root):
                    break
                if first.get((b, name)) == "setvar" and self._first_access_here(b, name):
                    self.local_vars.setdefault(b, set()).add(name)
                    break

    def _first_access_here(self, bid, name):
        """the first access of `name` in block bid's subtree (program order) is
        one of bid's own items"""
        blk = self._block_by_id(bid)
        for it in blk.items:
            if isinstance(it, (Loop, If)):
                if self._touches(it.body, name):
                    return False
            elif it.kind in ("getvar", "setvar") and it.imm == name:
                return it.kind == "setvar"
        return False

    def _touches(self, block, name):
        for it in block.items:
            if isinstance(it, (Loop, If)):
                if self._touches(it.body, name):
                    return True
            elif it.kind in ("getvar", "setvar") and it.imm == name:
                return True
        return False

    def _block_by_id(self, bid):
        if not hasattr(self, "_blocks"):
            self._blocks = {}

            def walk(b):
                self._blocks[id(b)] = b
                for it in b.items:
                    if isinstance(it, (Loop, If)):
                        walk(it.body)
            walk(self.prog.root)
        return self._blocks[bid]

    def block_vals(self, block):
        ids = {it.dst.id for it in block.items if isinstance(it, Op) and it.dst is not None}
        return ids | {it.dst2.id for it in block.items if isinstance(it, Op) and it.dst2 is not None}

    def park(self, block, pos):
        """before a construct: values of this block live after it leave the V
        slots (the body needs them all)"""
        self.wait_pending()
        ids = self.block_vals(block)
        for k in range(self.NV):
            vs = self.vslot[k]
            if vs is None or vs.val.id not in ids:
                continue
            if self.next_use(vs, pos) == 1 << 30:
                self.kill(vs)
                continue
            vs.locs.discard(("V", k))
            self.vslot[k] = None
            for loc in list(vs.locs):
                if loc in self.home.values():
                    vs.locs.discard(loc)
            if not vs.locs:
                loc = self.spill_slot(prefer="M")
                self.copy(("V", k), loc)
                self.own(loc, vs)
                vs.locs.add(loc)
                self.bump("park_" + loc[0])

    PRIO_TOGGLE = int(os.environ.get("PGEN_PRIO_TOGGLE", "0"))

    def run_construct(self, it):
        d = self.depth
        self.depth += 1
        w0 = self.weight
        if isinstance(it, Loop):
            self.weight = w0 * it.trips
            it.sreg = S_CNT + d
            top, done = self.label(), None
            self.i("s_mov_b32", S(it.sreg), K(it.trips - 1))
            self.i("label", top)
            if d == 0 and self.PRIO_TOGGLE:
                # A/B (PGEN_PRIO_TOGGLE=1): wave priority 2 in odd iterations of
                # the outer loop, 0 in even ones, so two co-resident waves of
                # one SIMD take turns instead of the older one keeping nearly
                # every issue slot (profiles/r05_coresidency.md)
                even, done_ = self.label(), self.label()
                self.i("s_and_b32", S(S_TMP), S(it.sreg), K(1))
                self.i("s_cmp_eq_u32", S(S_TMP), K(0))
                self.i("long_cbranch_scc1", even)
                self.i("s_setprio", self.PRIO_TOGGLE)
                self.i("s_cmp_eq_u32", S(S_TMP), S(S_TMP))
                self.i("long_cbranch_scc1", done_)
                self.i("label", even)
                self.i("s_setprio", 0)
                self.i("label", done_)
            self.untrack_stores()      # the previous iteration's stores
            self.run_block(it.body)
            self.i("s_sub_u32", S(it.sreg), S(it.sreg), K(1))
            self.i("s_cmp_ge_i32", S(it.sreg), K(0))
            self.i("long_cbranch_scc1", top)
            del done
        else:
            skip = self.label()
            m = S_MASK + 2 * d
            self.i("s_mov_b32", S(m), K(it.mask & 0xffffffff))
            self.i("s_mov_b32", S(m + 1), K(it.mask >> 32))
            self.i("s_bitcmp1_b64", S(m), S(it.loop.sreg))
            self.weight = w0 * bin(it.mask).count("1") / max(1, it.loop.trips)
            self.i("long_cbranch_scc0", skip)
            self.run_block(it.body)
            self.i("label", skip)
        if self.mstore:    # a skipped body: fewer operations in flight than counted
            self.untrack_stores()
        self.weight = w0
        self.depth -= 1

    def run_op(self, op, pos):
        k = op.kind
        self.bump("op_" + k)
        if k == "getvar":
            vs = self.states[op.dst.id]
            loc = self.home[op.imm]
            vs.locs.add(loc)
            vs.var = op.imm
            if not vs.uses:
                self.kill(vs)
            return
        if k == "setvar":
            self.do_setvar(op, pos)
            return
        srcs = [self.states[v.id] for v in op.srcs]
        self.pinned = set()
        sk = []
        self.defer_vm_wait = True
        for vs in srcs:
            kk = self.ensure_v(vs, pos, avoid=self.pinned)
            self.pinned.add(kk)
            sk.append(kk)
        self.defer_vm_wait = False
        if self.vm_wait_owed:
            # a demand reload stalls this operation: start the upcoming
            # operations' reloads first, so they travel during the same wait
            self.prefetch(pos, burst=True)
            self.vm_wait_owed = False
            self.wait_vm_count(min(63, self.vm_issued - self.vm_owed_seq))
        dying = [vs for vs in srcs if self.next_use(vs, pos) == 1 << 30]
        dk2 = None
        if op.dst2 is not None:
            # two-result ops (wsop, wnorm): fresh slots, no aliasing of sources
            dk = self.get_vslot(pos, avoid=self.pinned)
            self.pinned.add(dk)
            dk2 = self.get_vslot(pos, avoid=self.pinned)
            self.pinned.add(dk2)
        elif op.dst is not None:
            dvs = self.states[op.dst.id]
            # in place over a dying source (safe for every op kind below)
            dk = None
            for vs, kk in zip(srcs, sk):
                if (vs in dying and self.vslot[kk] is vs and k not in ("swap", "dppadd", "bcast", "pairz", "pdiff")
                        and not (k in ("sub", "csub") and op.srcs[0].id == op.srcs[1].id)):
                    dk = kk
                    break
            if dk is None:
                dk = self.get_vslot(pos, avoid=self.pinned)
        else:
            dk = None
        if any(x in self.pending for x in sk):
            self.wait_pending(sk)
        if dk2 is not None and dk2 in self.pending:
            self.wait_pending([dk2])
        if dk is not None:
            self.pinned.add(dk)
        scratch = []
        if k == "binv":
            for _ in range(4):
                kk = self.get_vslot(pos, avoid=self.pinned)
                self.pinned.add(kk)
                scratch.append(kk)
        self.prefetch(pos)
        base = [self.vbase(x) for x in sk]
        d = self.vbase(dk) if dk is not None else None
        if k == "sop":
            self.emit_sop(list(zip(base[0::2], base[1::2])), d)
        elif k == "sqr":
            self.emit_sop([(base[0], base[0])], d)
        elif k == "ssop":
            self.emit_sop([(base[0], base[1])], d, signed=True)
        elif k == "pdiff":
            self.emit_pdiff(base[0], d)
        elif k == "red":
            self.emit_red(base[0], d)
        elif k == "norm":
            self.emit_norm(base[0], d)
        elif k == "add":
            self.emit_add(base[0], base[1], d)
        elif k == "add3":
            for i in range(NL):
                self.i("v_add3_u32", d + i, base[0] + i, base[1] + i, base[2] + i)
        elif k == "shladd":
            for i in range(NL):
                self.i("v_lshl_add_u32", d + i, base[0] + i, K(op.imm), base[1] + i)
        elif k == "shl":
            for i in range(NL):
                self.i("v_lshlrev_b32", d + i, K(op.imm), base[0] + i)
        elif k == "sub":
            self.emit_sub(base[0], base[1], d, op.imm)
        elif k == "csub":
            self.emit_csub(base[0], base[1], d, op.imm)
        elif k == "wsop":
            self.emit_wsop(list(zip(base[0::2], base[1::2])), d, self.vbase(dk2))
        elif k == "wnorm":
            self.emit_wnorm(base[0], base[1], d, self.vbase(dk2))
        elif k == "wred":
            self.emit_wred(base[0], base[1], d)
        elif k == "neg":
            self.emit_neg(base[0], d, op.imm)
        elif k == "const":
            self.emit_const(op.imm, d)
        elif k == "swap":
            self.emit_swap(base[0], d)
        elif k == "sel":
            self.emit_sel(base[0], base[1], d)
        elif k == "bcast":
            self.emit_bcast(base[0], d, op.imm)
        elif k == "pairz":
            self.emit_pairz(base[0], d, op.imm)
        elif k == "dppadd":
            self.emit_dppadd(base[0], base[1], d, op.imm)
        elif k == "selz":
            nt = op.imm
            self.emit_selz(base[:nt], base[nt], base[nt + 1], d)
        elif k == "binv":
            self.emit_binv(base[0], d, scratch)
        elif k == "load_raw":
            self.cfg.emit_load(self, op.imm, d)
        elif k == "tload" and getattr(self.cfg, "per_lane_table", False):
            self.cfg.emit_tload(self, op.imm, d)
        elif k == "tnext" and getattr(self.cfg, "per_lane_table", False):
            self.cfg.emit_tnext(self)
        elif k == "tload":
            # every lane reads the same 56 bytes -- from the wave's LDS copy of
            # the table (a broadcast read; v17 = the line's LDS offset) or from
            # global memory (one cache line request per load); the value is
            # used after the line's other loads are issued, so the wait is a
            # counted one at its first use (self.pending)
            for j in range(7):
                if getattr(self.cfg, "lds_table", False):
                    self.i("ds_read_b64", d + 2 * j, ZERO, NL * 4 * op.imm + 8 * j)
                else:
                    self.i("global_load_dwordx2_s", d + 2 * j, ZERO, S(S_LINE), NL * 4 * op.imm + 8 * j)
        elif k == "tnext":
            if getattr(self.cfg, "lds_table", False):
                self.i("v_add_u32", ZERO, K(LINE_BYTES), ZERO)
            else:
                self.i("s_add_u32", S(S_LINE), S(S_LINE), K(LINE_BYTES))
                self.i("s_addc_u32", S(S_LINE + 1), S(S_LINE + 1), K(0))
        elif k == "store_raw":
            self.cfg.emit_store(self, op.imm, base[0])
        else:
            raise AllocError(k)
        self.pinned = set()
        for vs in dying:
            # the destination may have taken its V slot
            for loc in list(vs.locs):
                if loc[0] == "V" and loc[1] in (dk, dk2):
                    vs.locs.discard(loc)
                    continue
                self.release_loc(loc, vs)
            vs.locs.clear()
        for dst, kk in ((op.dst, dk), (op.dst2, dk2)):
            if dst is None:
                continue
            dvs = self.states[dst.id]
            self.vslot[kk] = dvs
            dvs.locs = {("V", kk)}
            if k == "tload":
                lds = getattr(self.cfg, "lds_table", False) or getattr(self.cfg, "per_lane_table", False)
                self.pending[kk] = ("L", self.lgkm_issued) if lds else ("M", self.vm_issued)
                if getattr(self.cfg, "per_lane_table", False):
                    self.split_pending[kk] = True
            if self.debug and k != "tload":   # a table load lands at its counted wait
                self.i("mark", dst.id, self.vbase(kk))
            if not dvs.uses:
                self.kill(dvs)

    # ---------------- prefetch ----------------
    COST = {"sop": None, "sqr": 460, "red": 62, "norm": 39, "add": 14, "add3": 14, "shladd": 14, "shl": 14, "sub": 28, "neg": 14, "const": 14, "swap": 15,
            "sel": 14, "dppadd": 15, "bcast": 15, "pairz": 29, "pdiff": 31, "load_raw": 60, "store_raw": 200, "getvar": 0, "setvar": 14, "tload": 7, "tnext": 2,
            "selz": 80, "binv": 33000}
    # instructions of other work that hide the load latency (PGEN_AHEAD_L/_M: experiments)
    AHEAD = {"L": int(os.environ.get("PGEN_AHEAD_L", 40)), "M": int(os.environ.get("PGEN_AHEAD_M", 500))}
    WINDOW = int(os.environ.get("PGEN_WINDOW", 2500))

    def op_cost(self, op):
        if op.kind == "ssop":
            return 196 * 2 + 71
        if op.kind == "sop":
            return 196 * (len(op.srcs) // 2 + 1) + 70
        if op.kind == "wsop":
            return 196 * (len(op.srcs) // 2) + 60
        if op.kind == "wred":
            return 260
        if op.kind in ("csub", "wnorm"):
            return 28 if op.kind == "csub" else 84
        return self.COST.get(op.kind, 20)

    def prefetch(self, pos, burst=False):
        """issue the LDS / HBM reloads of upcoming operations now, so their
        latency hides behind the current operation's arithmetic (burst: HBM
        reloads of the next few operations however close, while this one
        waits for its own)"""
        items = self.items
        work = 0
        for j in range(pos, min(len(items), pos + 40)):
            it = items[j]
            if not isinstance(it, Op):
                break
            if j > pos:
                for v in it.srcs:
                    vs = self.states.get(v.id)
                    if vs is None or any(l[0] == "V" for l in vs.locs) or not vs.locs:
                        continue
                    src = self.best_src(vs)
                    if src[0] == "A" or (work < self.AHEAD[src[0]] and not (burst and src[0] == "M")):
                        continue
                    k = self.prefetch_slot(pos, j)
                    if k is None:
                        return
                    self.copy(src, ("V", k), wait=False)
                    self.vslot[k] = vs
                    vs.locs.add(("V", k))
                    self.pending[k] = (src[0], self.lgkm_issued if src[0] == "L" else self.vm_issued)
                    self.bump("prefetch_" + src[0])
            work += self.op_cost(it)
            if work > (self.AHEAD["M"] if burst else self.WINDOW):
                break

    def prefetch_slot(self, pos, j):
        """a V slot whose value is not needed before op j (free, or evictable)"""
        for k in range(self.NV):
            if self.vslot[k] is None and k not in self.pinned and k not in self.pending:
                return k
        best, bk = j, None
        for k in range(self.NV):
            if k in self.pinned or k in self.pending or self.vslot[k] is None:
                continue
            if len(self.vslot[k].locs) < 2:
                continue    # dirty: evicting it would cost a spill
            nu = self.next_use(self.vslot[k], pos)
            if nu > best:
                best, bk = nu, k
        if bk is None:
            return None
        self.evict(bk, pos)
        return bk

    def do_setvar(self, op, pos):
        name = op.imm
        vs = self.states[op.srcs[0].id]
        home = self.home[name]
        if home[0] == "V":
            raise AllocError("V homes unsupported")
        # values still holding the old contents of this home keep a copy
        for other in list(self.states.values()):
            if other is not vs and home in other.locs:
                if len(other.locs) == 1 and self.next_use(other, pos) != 1 << 30:
                    self.ensure_v(other, pos, avoid=())
                other.locs.discard(home)
        if home not in vs.locs:
            k = self.ensure_v(vs, pos, avoid=())
            if k in self.pending:
                self.wait_pending([k])
            self.copy(("V", k), home)
        if self.next_use(vs, pos) == 1 << 30:
            self.kill(vs)
