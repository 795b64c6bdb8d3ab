"""Kernel-level glue for the generated kernels: argument layout, prologue,
record loads / canonical stores, the lane masks for infinity (Miller loop)
and f == 0 (final exponentiation), epilogue.

Kernel arguments (5 x 8 bytes, all kernels):
  miller_loop: p_aff (G1Affine, 13 u64), q_aff (G2Affine, 25 u64), out (Fq12, 72 u64), n, workspace
  final_exp:   in (Fq12), out (Fq12), ok (u8 per lane, may be null), n, workspace
"""
import os

import gen_fl
from dsl import Q
from emit import (A, ACC, ADDR, GID, K, LOFF, ORACC, S, S_ARG, S_EXEC, S_KARG, S_LINE, S_ODD, S_TMP, S_VALID,
                  S_WG, S_WS, SKQ, SQ, SQINV, NL, MASK, QL, QINV28, KQ, ZERO)

ONE_ABI = (1 << 384) % Q          # Montgomery one in the ABI (R = 2^384)
S_STRIDE = 32


def words32(x, n=12):
    return [(x >> (32 * j)) & 0xffffffff for j in range(n)]


class KernelCfg:
    """lanes = 1: lane i handles pairing i.  lanes = 2: lanes 2j and 2j+1
    handle pairing j (role r = lane & 1); a load / store slot pair (s0, s1)
    means lane r uses slot s_r of pairing j's record."""
    name = None
    lanes = 1
    args = ()
    records = {}          # input slot -> (arg index, record bytes, byte offset)
    out_arg, out_bytes = 2, 576

    def emit_prologue(self, em, code, nmem, end_label):
        i = code.append
        for a in range(5):
            i(("s_load_dwordx2", S(S_ARG + 2 * a), S(S_KARG), 8 * a))
        i(("s_waitcnt_lgkm0",))
        i(("v_lshlrev_b32", LOFF, K(3), 0))
        i(("v_lshl_add_u32", GID, S(S_WG), K(6), 0))   # global lane index
        if self.lanes == 2:
            i(("s_lshl_b32", S(S_ARG + 6), S(S_ARG + 6), K(1)))   # 2n active lanes
            i(("s_mov_b32", S(S_ODD), K(0xAAAAAAAA)))
            i(("s_mov_b32", S(S_ODD + 1), K(0xAAAAAAAA)))
        self.pre_exec(em, code)
        i(("v_cmp_gt_u32", S(S_ARG + 6), GID))
        i(("s_and_saveexec_b64", S(S_EXEC)))
        i(("long_cbranch_execz", end_label))
        for k, w in enumerate(QL):
            i(("s_mov_b32", S(SQ + k), K(w)))
        i(("s_mov_b32", S(SQINV), K(QINV28)))
        i(("s_mov_b32", S(SKQ), K(KQ)))
        for sreg, v in em.ctab_init:
            i(("s_mov_b32", S(sreg), K(v)))
        wave_bytes = max(nmem, 1) * gen_fl.NL * 4 * 64
        i(("s_mul_i32", S(S_TMP), S(S_WG), K(wave_bytes)))
        i(("s_mul_hi_u32", S(S_TMP + 1), S(S_WG), K(wave_bytes)))
        i(("s_add_u32", S(S_WS), S(S_ARG + 8), S(S_TMP)))
        i(("s_addc_u32", S(S_WS + 1), S(S_ARG + 9), S(S_TMP + 1)))
        self.prologue_masks(em, code)

    def prologue_masks(self, em, code):
        pass

    def pre_exec(self, em, code):
        """work every lane of the wave does before the lanes past n are masked off"""
        pass

    nl = None          # LDS spill slots of this kernel (None: emit.STORAGE)
    extra_lds = 0      # LDS bytes behind the spill slots (a staged table)

    def lane_addr(self, code, arg, stride, delta=0):
        """v[12:13] = arg + (pairing index) * stride + (lane role) * delta"""
        # global lane index from tid * 8; one SGPR per VALU instruction
        # (constant bus): the base goes through VGPRs
        code.append(("v_lshrrev_b32", GID, K(3), LOFF))
        code.append(("v_lshl_add_u32", GID, S(S_WG), K(6), GID))
        if self.lanes == 2:
            code.append(("v_and_b32", 15, K(1), GID))
            code.append(("v_lshrrev_b32", GID, K(1), GID))
        code.append(("v_mov_b64", ADDR, S(S_ARG + 2 * arg)))
        code.append(("s_mov_b32", S(S_STRIDE), K(stride)))
        code.append(("v_mad_u64_u32", ADDR, GID, S(S_STRIDE), ADDR))
        if self.lanes == 2 and delta:
            code.append(("v_mul_u32_u24", 15, K(delta), 15))
            code.append(("v_mad_u64_u32", ADDR, 15, K(1), ADDR))

    def slot_pair(self, imm):
        return imm if isinstance(imm, tuple) else (imm, imm)

    def emit_load(self, em, slot, d):
        s0, s1 = self.slot_pair(slot)
        arg, stride, off = self.records[s0]
        arg1, stride1, off1 = self.records[s1]
        assert (arg, stride) == (arg1, stride1)
        self.lane_addr(em.code, arg, stride, off1 - off)
        for j in range(6):
            em.i("global_load_dwordx2", 2 * j, ADDR, off + 8 * j)
        em.i("s_waitcnt_vm0")
        self.after_load(em, slot)
        for li in range(NL):
            bit = 28 * li
            wi, sh = bit // 32, bit % 32
            if wi + 1 < 12:
                em.i("v_alignbit_b32", d + li, wi + 1, wi, K(sh))
                em.i("v_and_b32", d + li, K(MASK), d + li)
            else:
                em.i("v_lshrrev_b32", d + li, K(sh), wi)

    def after_load(self, em, slot):
        pass

    def emit_store(self, em, slot, t):
        # canonical: t (limbs < 2^28, value < 2q) -> t mod q, in place
        bor = 14
        for li in range(NL):
            em.i("v_subrev_u32", li, K(QL[li]), t + li)
            if li:
                em.i("v_add_u32", li, li, bor)
            em.i("v_ashrrev_i32", bor, K(28), li)
            em.i("v_and_b32", li, K(MASK), li)
        for li in range(NL):
            em.i("v_bfi_b32", t + li, bor, t + li, li)   # t < q ? t : t - q
        # pack 14 x 28 -> 12 x 32 into v0..v11
        for j in range(12):
            bit = 32 * j
            li, sh = bit // 28, bit % 28
            em.i("v_lshrrev_b32", j, K(sh), t + li)
            em.i("v_lshl_or_b32", j, t + li + 1, K(28 - sh), j)
            if 56 - sh < 32 and li + 2 < NL:
                em.i("v_lshl_or_b32", j, t + li + 2, K(56 - sh), j)
        # lanes that are not valid get the fixed value
        s0, s1 = self.slot_pair(slot)
        em.i("s_mov_b64", S(106), S(S_VALID))
        em.i("s_nop", 1)
        for j, (w0, w1) in enumerate(zip(self.invalid_words(s0), self.invalid_words(s1))):
            if w0 == w1 and -16 <= w0 <= 64:    # inline constant: no constant-bus slot
                em.i("v_cndmask_b32", j, K(w0), j)
                continue
            em.i("v_mov_b32", 15, K(w0))            # literal + VCC would need two
            if w1 != w0:
                em.i("v_mov_b32", 14, K(w1))
                em.i("v_cndmask_b32_e64", 15, 15, 14, S(S_ODD))
            em.i("v_cndmask_b32", j, 15, j)
        self.lane_addr(em.code, self.out_arg, self.out_bytes, 48 * (s1 - s0))
        for j in range(6):
            em.i("global_store_dwordx2", ADDR, 2 * j, 48 * s0 + 8 * j)

    def invalid_words(self, slot):
        raise NotImplementedError

    def emit_epilogue(self, em, code):
        pass


class MillerLoopCfg(KernelCfg):
    name = "pa_gen_miller_loop"
    records = {0: (0, 104, 0), 1: (0, 104, 48),
               2: (1, 200, 0), 3: (1, 200, 48), 4: (1, 200, 96), 5: (1, 200, 144)}

    def prologue_masks(self, em, code):
        # valid = neither P nor Q is the point at infinity (mod.rs:50-54)
        self.lane_addr(code, 0, 104)
        code.append(("global_load_dword", 0, ADDR, 96))
        self.lane_addr(code, 1, 200)
        code.append(("global_load_dword", 1, ADDR, 192))
        code.append(("s_waitcnt_vm0",))
        code.append(("v_or_b32", 0, 0, 1))
        code.append(("v_and_b32", 0, K(0xff), 0))
        code.append(("v_cmp_eq_u32", K(0), 0))
        code.append(("s_nop", 1))
        code.append(("s_mov_b64", S(S_VALID), S(106)))

    def invalid_words(self, slot):
        # one (fq12.rs): only coordinate 0 is one
        return words32(ONE_ABI) if slot == 0 else [0] * 12


class FinalExpCfg(KernelCfg):
    name = "pa_gen_final_exp"
    # slot 12 (split final exponentiation, "inv" program): the inverted norm
    # that the "norm" program stored as Fq 0 of the out record
    records = {**{k: (0, 576, 48 * k) for k in range(12)}, 12: (1, 576, 0)}
    out_arg = 1

    def prologue_masks(self, em, code):
        code.append(("v_mov_b32", ORACC, K(0)))

    def after_load(self, em, slot):
        for j in range(12):
            em.i("v_or_b32", ORACC, ORACC, j)
        if self.slot_pair(slot)[1] == 11:
            if self.lanes == 2:   # the pair's two halves of the record
                em.i("s_nop", 1)
                em.i("v_mov_b32_dpp_swap", 14, ORACC)
                em.i("v_or_b32", ORACC, ORACC, 14)
            em.i("v_cmp_ne_u32", K(0), ORACC)
            em.i("s_nop", 1)
            em.i("s_mov_b64", S(S_VALID), S(106))

    def invalid_words(self, slot):
        return [0] * 12      # reference: None; the C ABI writes zero and ok = 0

    def emit_epilogue(self, em, code):
        skip = em.label()
        code.append(("s_cmp_eq_u64", S(S_ARG + 4), K(0)))
        code.append(("long_cbranch_scc1", skip))
        code.append(("v_mov_b32", 1, K(1)))
        code.append(("s_mov_b64", S(106), S(S_VALID)))
        code.append(("s_nop", 1))
        code.append(("v_cndmask_b32", 0, K(0), 1))
        self.lane_addr(code, 2, 1)
        code.append(("global_store_byte", ADDR, 0, 0))
        code.append(("label", skip))


class MillerLoopSharedCfg(MillerLoopCfg):
    """miller_loop of every P_i against ONE G2Prepared (kernels.
    miller_loop_shared_prog).  Arguments: p_aff (G1Affine records), table,
    out (Fq12), n, workspace.  The table (written by k_shared_line_table,
    kernels_pairing.hip) is u32 words: word 0 = Q's infinity flag, then from
    byte TABLE_LINES the 68 lines of six 14-limb values (22 848 B).

    LDS staging (default): every wave copies the lines into its LDS behind
    its five spill slots before masking the lanes past n (45 coalesced 512-byte
    rows), and the loop reads them with ds_read_b64 at a wave-uniform address
    (v17 = the current line's LDS offset; all lanes read the same words, a
    broadcast).  4 waves x (5 x 3584 + 23 040) B = 160 KiB per CU.
    PGEN_MLS_LDS=0: read the table from global memory instead (wave-uniform
    global_load_dwordx2 with v17 = 0 and the line pointer in s[96:97])."""
    name = "pa_gen_miller_loop_shared"
    records = {0: (0, 104, 0), 1: (0, 104, 48)}
    TABLE_LINES = 64
    TABLE_ROWS = 45                      # 45 x 512 B >= 68 x 336 B
    nsgpr = 98          # s[96:97]: the line pointer (global form)

    def __init__(self):
        import os
        self.lds_table = os.environ.get("PGEN_MLS_LDS", "1") == "1"
        if self.lds_table:
            self.nl = 5
            self.extra_lds = 512 * self.TABLE_ROWS

    def table_base(self):
        return self.nl * gen_fl.NL * 4 * 64

    def pre_exec(self, em, code):
        if not self.lds_table:
            return
        i = code.append
        # rows of 512 B (8 B per lane) from the global table into LDS, seven
        # loads in flight at a time (v0..v13), offsets within 4 KiB of s[16:17]
        for b0 in range(0, self.TABLE_ROWS, 7):
            rows = range(b0, min(b0 + 7, self.TABLE_ROWS))
            i(("s_add_u32", S(S_TMP), S(S_ARG + 2), K(self.TABLE_LINES + 512 * b0)))
            i(("s_addc_u32", S(S_TMP + 1), S(S_ARG + 3), K(0)))
            for k, r in enumerate(rows):
                i(("global_load_dwordx2_s", 2 * k, LOFF, S(S_TMP), 512 * (r - b0)))
            i(("s_waitcnt_vm0",))
            for k, r in enumerate(rows):
                i(("ds_write_b64", LOFF, 2 * k, self.table_base() + 512 * r))
        i(("s_waitcnt_lgkm0",))

    def prologue_masks(self, em, code):
        i = code.append
        # valid = P is not the point at infinity and Q is not (the table's flag)
        i(("v_mov_b32", ZERO, K(0)))
        self.lane_addr(code, 0, 104)
        i(("global_load_dword", 0, ADDR, 96))
        i(("global_load_dwordx2_s", 2, ZERO, S(S_ARG + 2), 0))
        i(("s_waitcnt_vm0",))
        i(("v_or_b32", 0, 0, 2))
        i(("v_and_b32", 0, K(0xff), 0))
        i(("v_cmp_eq_u32", K(0), 0))
        i(("s_nop", 1))
        i(("s_mov_b64", S(S_VALID), S(106)))
        if self.lds_table:
            i(("v_mov_b32", ZERO, K(self.table_base())))
        else:
            i(("s_add_u32", S(S_LINE), S(S_ARG + 2), K(self.TABLE_LINES)))
            i(("s_addc_u32", S(S_LINE + 1), S(S_ARG + 3), K(0)))


class MillerLoopPreparedCfg(MillerLoopSharedCfg):
    """miller_loop of (P_i, G2Prepared_i) pairs (kernels.miller_loop_prepared_prog).
    Arguments: p_aff (G1Affine records), prepared (G2Prepared records of
    RECORD bytes: 68 lines of (c0, c1, c2) Fq2 in the ABI form, the infinity
    flag at FLAG), out (Fq12), n, workspace.

    The wave copies the current line of its 64 records (64 x 288 B) into an
    LDS buffer one line AHEAD, with 18 global_load_lds_dwordx4: slot s = tid +
    64 t of copy t is piece s % 18 (16 B) of record s / 18, so the buffer holds
    record r's line at 288 r and every copy instruction reads 4-5 contiguous
    288-byte runs -- not 64 records 19.6 KB apart (measured at 2^16: 6.53 ms
    against 6.66 for the per-lane scatter).  What the copy still costs (6.07
    ms with no copy at all, 6.15 with every lane copying one address) is not
    its latency: waiting for it right after issue costs 0.08 ms more, not
    waiting at all (wrong results) nothing less, and L2-resident source lines
    (line 0 every time) 0.05 ms less.  The copy runs with every lane
    of the wave on (the record index clamped to n - 1), since lanes past n
    still copy pieces for lanes below it.

    tnext (after the line's values are in registers) waits for the buffer's
    reads and issues the next line's copy, which lands under mul_by_014 and the
    squaring; the first tload of a line waits for it (vmcnt 0); each value is
    read with ds_read_b64 at v17 = 288 tid and split into its 14 limbs when it
    lands (emit_split).  s[96] = the line's byte offset in a record; the copy
    after the last line re-reads line 67 (s[97] = min(s[96], 67 lines)).  LDS
    per wave: five spill slots + the 18 KiB buffer (36 352 B; four waves per
    CU).  s[98:99] exec saved around a copy, s100 = n - 1, s101 = the wave's
    first record."""
    name = "pa_gen_miller_loop_prepared"
    RECORD, FLAG, LINE = 19592, 19584, 288
    PIECES = 18                 # 288 B per lane / 16 B per global_load_lds_dwordx4
    nsgpr = 102

    def __init__(self):
        self.lds_table = False
        self.per_lane_table = True
        self.nl = 5
        self.extra_lds = 1024 * self.PIECES

    def pre_exec(self, em, code):
        pass

    def emit_copy(self, put):
        """line s[97] of the wave's 64 records -> the LDS buffer (in flight)"""
        put("wave_begin")                               # simulator: every lane runs the copy
        put("s_or_saveexec_b64", S(98), K(-1))
        put("v_lshrrev_b32", 3, K(3), LOFF)             # tid
        for t in range(self.PIECES):
            put("v_add_u32", 0, K(64 * t), 3)           # slot s
            put("v_mul_u32_u24", 1, K(3641), 0)
            put("v_lshrrev_b32", 1, K(16), 1)           # r = s / 18 (exact for s < 1152)
            put("v_mul_u32_u24", 2, K(18), 1)
            put("v_sub_u32", 2, 0, 2)                   # piece j = s - 18 r
            put("v_add_u32", 1, S(101), 1)
            put("v_min_u32", 1, S(100), 1)              # record, clamped to n - 1
            put("v_lshlrev_b32", 2, K(4), 2)
            put("v_add_u32", 2, S(S_LINE + 1), 2)       # byte offset in the record
            put("v_mov_b64", ADDR, S(S_ARG + 2))
            put("v_mad_u64_u32", ADDR, 1, S(S_STRIDE), ADDR)
            put("v_mad_u64_u32", ADDR, 2, K(1), ADDR)
            put("s_mov_m0", K(self.table_base() + 1024 * t))
            put("s_nop", 0)
            put("global_load_lds_dwordx4", ADDR)
        put("s_mov_b64_exec", S(98))
        put("wave_end")

    def prologue_masks(self, em, code):
        i = code.append
        # valid = neither P nor this lane's prepared Q is the point at infinity
        self.lane_addr(code, 0, 104)
        i(("global_load_dword", 0, ADDR, 96))
        self.lane_addr(code, 1, self.RECORD)
        i(("v_mov_b32", 14, K(self.FLAG)))
        i(("v_mad_u64_u32", ADDR, 14, K(1), ADDR))
        i(("global_load_dword", 1, ADDR, 0))
        i(("s_waitcnt_vm0",))
        i(("v_or_b32", 0, 0, 1))
        i(("v_and_b32", 0, K(0xff), 0))
        i(("v_cmp_eq_u32", K(0), 0))
        i(("s_nop", 1))
        i(("s_mov_b64", S(S_VALID), S(106)))
        i(("v_mul_u32_u24", ZERO, K(36), LOFF))          # 288 tid: this lane's line in the buffer
        i(("s_mov_b32", S(S_LINE), K(0)))
        i(("s_mov_b32", S(S_LINE + 1), K(0)))
        i(("s_sub_u32", S(100), S(S_ARG + 6), K(1)))
        i(("s_lshl_b32", S(101), S(S_WG), K(6)))
        i(("s_mov_b32", S(S_STRIDE), K(self.RECORD)))
        self.emit_copy(lambda *t: i(t))                  # line 0

    def emit_tload(self, em, imm, d):
        """value imm of the current line: its 12 words from the LDS buffer into
        d..d+11, in flight (a counted lgkm wait and the split at first use)"""
        if imm == 0:
            em.i("s_waitcnt_vm0")      # the line's copy has landed
        for j in range(6):
            em.i("ds_read_b64", d + 2 * j, ZERO, self.table_base() + 48 * imm + 8 * j)

    @staticmethod
    def emit_split(em, d):
        """12 x 32-bit words in d..d+11 -> 14 x 28-bit limbs in d..d+13, in place:
        limb k reads words <= k only, so from the top limb down"""
        for li in reversed(range(NL)):
            bit = 28 * li
            wi, sh = bit // 32, bit % 32
            if sh == 0:
                em.i("v_and_b32", d + li, K(MASK), d + wi)
            elif sh + 28 == 32 or wi + 1 == 12:     # the limb's top bits end the word
                em.i("v_lshrrev_b32", d + li, K(sh), d + wi)
            else:
                em.i("v_alignbit_b32", d + li, d + wi + 1, d + wi, K(sh))
                em.i("v_and_b32", d + li, K(MASK), d + li)

    def emit_tnext(self, em):
        em.i("s_waitcnt_lgkm0")        # this line's reads of the buffer are done
        em.i("s_add_u32", S(S_LINE), S(S_LINE), K(self.LINE))
        em.i("s_min_u32", S(S_LINE + 1), S(S_LINE), K(self.FLAG - self.LINE))
        em.i("s_mov_b32", S(S_STRIDE), K(self.RECORD))
        self.emit_copy(em.i)


class MillerLoopCfg2(MillerLoopCfg):
    name = "pa_gen_miller_loop2"
    lanes = 2


class MillerLoopCfg2p(MillerLoopCfg2):
    """the pairing-only lane-pair Miller loop (kernels.miller_loop_prog(pairing_only=True)):
    same records, masks and output slots as MillerLoopCfg2"""
    name = "pa_gen_miller_loop2p"


class MillerLoopCfg1p(MillerLoopCfg):
    """the pairing-only one-lane Miller loop (kernels.miller_loop_prog(pairing_only=True)):
    same records, masks and output slots as MillerLoopCfg"""
    name = "pa_gen_miller_loop1p"


class FinalExpCfg2(FinalExpCfg):
    name = "pa_gen_final_exp2"
    lanes = 2


def build(prog, cfg, debug=False):
    """allocate + emit: returns (code list, emitter)"""
    import os
    from emit import Emitter, plan_ctab
    from dsl import fuse_adds
    if prog.use_norm and os.environ.get("PGEN_FUSE", "1") == "1":
        fuse_adds(prog)
    plan = None
    if os.environ.get("PGEN_SAD", "1") == "1":
        # first pass: which subtraction constants the program uses, how often
        em0 = Emitter(prog, cfg)
        em0.run_block(prog.root, top=True)
        plan = plan_ctab(em0.sub_hist)
    em = Emitter(prog, cfg, plan)
    em.debug = debug
    em.run_block(prog.root, top=True)
    body = em.code
    code = []
    end = em.label()
    cfg.emit_prologue(em, code, len(em.mslot), end)
    code.extend(body)
    cfg.emit_epilogue(em, code)
    code.append(("label", end))
    code.append(("s_endpgm",))
    em.code = code
    em.lds_bytes = len(em.lslot) * gen_fl.NL * 4 * 64 + cfg.extra_lds
    return code, em
