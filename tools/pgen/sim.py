"""Single-lane simulator of the instruction subset emit.py / kcfg.py produce.

Executes the abstract instruction list (before text rendering) for one lane
with a 256 VGPR / 256 AGPR / 108 SGPR register file, byte-addressed global
memory and per-lane LDS, so register-allocation or emission bugs show up on
the CPU as a difference against dsl.evaluate.
"""
M32 = 0xffffffff
M64 = (1 << 64) - 1


def sx32(x):
    x &= M32
    return x - (1 << 32) if x >> 31 else x


def sx64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


class Sim:
    """lanes: the simulated lanes (one, or the two lanes of a pair); VALU /
    memory instructions run per lane, SALU once, DPP reads the partner."""

    def __init__(self, code, lane=0, lanes=None):
        self.code = code
        self.lanes = lanes or [lane]
        self.inflight = {}   # (lane, vgpr) -> ("lgkm" | "vm", seq, value): loads not yet waited for
        self.seq = {"lgkm": 0, "vm": 0}
        self.st_inflight = {}  # dword address -> vm seq of a workspace store not yet waited for
        self.vf = {ln: [0] * 256 for ln in self.lanes}
        self.af = {ln: [0] * 256 for ln in self.lanes}
        self.v = self.vf[self.lanes[0]]
        self.a = self.af[self.lanes[0]]
        self.s = [0] * 108
        self.scc = 0
        self.mem = {}       # dword address -> u32
        self.lds = {}
        self.lds_dma = {}     # LDS byte address -> (vm seq, word): global_load_lds data not yet waited for
        self.m0 = 0
        self.lane = lane
        self.labels = {t[1]: i for i, t in enumerate(code) if t[0] == "label"}
        self.count = 0
        self.hist = {}
        self.trace = None
        self.ws = 0              # wait-state clock: +1 per instruction, +N+1 per s_nop N
        self.sgpr_vwrite = {}    # SGPR number -> wait-state clock of its last VALU write

    # gfx950: a VALU read of an SGPR (mask, carry-in or operand) must come two
    # wait states after a VALU instruction wrote it (LLVM inserts s_nop 1 there)
    VALU_SW = {"v_mad_u64_u32": "vcc", "v_mad_i64_i32": "vcc", "v_sub_co_u32": "vcc", "v_subb_co_u32": "vcc"}
    VALU_SR = {"v_cndmask_b32": "vcc", "v_subb_co_u32": "vcc", "v_cndmask_b32_dpp_swap": "vcc"}

    def hazard(self, t):
        m, a = t[0], t[1:]
        if not m.startswith("v_"):
            return
        reads = set()
        if m in self.VALU_SR:
            reads.add(106)
        if m.startswith("v_cmp") and not m.endswith("_e64"):
            srcs = a
        elif m.startswith("v_cmp"):
            srcs = a[1:]
        else:
            srcs = a[1:]
        for x in srcs:
            if isinstance(x, int) and x >= 512:
                reads.add(x - 512)
        for r in reads:
            for rr in (r, r + 1):
                w = self.sgpr_vwrite.get(rr)
                if w is not None and self.ws - w - 1 < 2:
                    raise AssertionError("VALU read of s%d %d wait states after a VALU write (instr %d: %r)" % (
                        rr, self.ws - w - 1, self.count, t))
        writes = []
        if m in self.VALU_SW or (m.startswith("v_cmp") and not m.endswith("_e64")):
            writes.append(106)
        elif m.startswith("v_cmp"):
            writes.append(a[0] - 512)
        for r in writes:
            self.sgpr_vwrite[r] = self.sgpr_vwrite[r + 1] = self.ws

    # ---------- operand access ----------
    def chk(self, x):
        if (self.lane, x) in self.inflight:
            raise AssertionError("v%d read/overwritten before its load was waited for (instr %d: %r)" % (
                x, self.count, self.code[self.pc]))

    def rd(self, x):
        if isinstance(x, tuple):
            return x[1] & M32
        if x < 256 and self.inflight:
            self.chk(x)
        if x >= 512:
            return self.s[x - 512]
        if x >= 256:
            return self.a[x - 256]
        return self.v[x]

    def rd64(self, x):
        if isinstance(x, tuple):
            return x[1] & M64
        if x < 256 and self.inflight:
            self.chk(x)
            self.chk(x + 1)
        if x >= 512:
            return self.s[x - 512] | (self.s[x - 511] << 32)
        return self.v[x] | (self.v[x + 1] << 32)

    def wr(self, x, val):
        val &= M32
        if x < 256 and self.inflight:
            self.chk(x)
        if x >= 512:
            self.s[x - 512] = val
        elif x >= 256:
            self.a[x - 256] = val
        else:
            self.v[x] = val

    def wr64(self, x, val):
        self.wr(x, val & M32)
        self.wr(x + 1, (val >> 32) & M32)

    def set_vcc(self, bit):
        m = self.s[106] | (self.s[107] << 32)
        b = self.lane % 64
        m = (m & ~(1 << b)) | (int(bool(bit)) << b)
        self.s[106], self.s[107] = m & M32, m >> 32

    def vcc_of(self, ln):
        m = self.s[106] | (self.s[107] << 32)
        return (m >> (ln % 64)) & 1

    def vcc(self):
        m = self.s[106] | (self.s[107] << 32)
        return (m >> (self.lane % 64)) & 1

    def set_mask(self, sreg, bit):
        """lane bit of a 64-bit SGPR-pair mask (sreg: operand number >= 512)"""
        n = sreg - 512
        m = self.s[n] | (self.s[n + 1] << 32)
        b = self.lane % 64
        m = (m & ~(1 << b)) | (int(bool(bit)) << b)
        self.s[n], self.s[n + 1] = m & M32, m >> 32

    def mask_bit(self, sreg):
        n = sreg - 512
        return ((self.s[n] | (self.s[n + 1] << 32)) >> (self.lane % 64)) & 1

    def async_wr(self, kind, x, val):
        if self.inflight:
            self.chk(x)
        self.inflight[(self.lane, x)] = (kind, self.seq[kind], val & M32)

    def complete(self, kind, keep=0):
        """s_waitcnt <kind>(keep): all but the `keep` youngest operations are done"""
        limit = self.seq[kind] - keep
        if kind == "vm":
            for ad in [ad for ad, sq in self.st_inflight.items() if sq <= limit]:
                del self.st_inflight[ad]
        if kind == "vm":
            for ad in [ad for ad, (sq, _) in self.lds_dma.items() if sq <= limit]:
                self.lds[ad] = self.lds_dma.pop(ad)[1]
        for key in [k for k, (kd, sq, _) in self.inflight.items() if kd == kind and sq <= limit]:
            ln, x = key
            self.vf[ln][x] = self.inflight.pop(key)[2]

    def ld32(self, addr):
        return self.mem.get(addr, 0)

    def st32(self, addr, val):
        self.mem[addr] = val & M32

    # ---------- execution ----------
    def run(self, max_steps=10 ** 9):
        code = self.code
        pc = 0
        n = len(code)
        while pc < n:
            self.pc = pc
            t = code[pc]
            if t[0] == "wave_begin":
                pc = self.run_wave(pc)
                continue
            self.count += 1
            if self.count > max_steps:
                raise RuntimeError("step limit")
            m = t[0]
            self.hist[m] = self.hist.get(m, 0) + 1
            self.hazard(t)
            self.ws += (t[1] + 1) if m == "s_nop" else 1
            if m.startswith("ds_"):
                self.seq["lgkm"] += 1
            elif m.startswith("global_"):
                self.seq["vm"] += 1
            if m.startswith("v_") or m.startswith("ds_") or m.startswith("global_") or m == "mark":
                if m == "v_mov_b32_dpp_swap":
                    src = {ln: self.vf[ln][t[2]] for ln in self.lanes}
                    for ln in self.lanes:
                        self.vf[ln][t[1]] = src[ln ^ 1] if (ln ^ 1) in src else 0
                    nxt = None
                elif m == "v_mov_b32_dpp_bcast":
                    src = {ln: self.vf[ln][t[2]] for ln in self.lanes}
                    for ln in self.lanes:
                        self.vf[ln][t[1]] = src[(ln & ~1) | t[3]]
                    nxt = None
                elif m == "v_sub_u32_dpp_bcast0":
                    # lane ln: src0 of the pair's lane 0 minus its own src1
                    src = {ln: self.vf[ln][t[2]] for ln in self.lanes}
                    val = {ln: (src[ln & ~1] - self.vf[ln][t[3]]) & 0xffffffff for ln in self.lanes}
                    for ln in self.lanes:
                        self.vf[ln][t[1]] = val[ln]
                    nxt = None
                elif m == "v_cndmask_b32_dpp_swap":
                    # lane ln: VCC ? its own src1 : src0 of its partner lane
                    src = {ln: self.vf[ln][t[2]] for ln in self.lanes}
                    val = {ln: self.vf[ln][t[3]] if self.vcc_of(ln) else (src[ln ^ 1] if (ln ^ 1) in src else 0)
                           for ln in self.lanes}
                    for ln in self.lanes:
                        self.vf[ln][t[1]] = val[ln]
                    nxt = None
                elif m == "v_add_u32_dpp":
                    # lane ln reads src0 from lane (ln & ~1) | perm[ln & 1] of its pair
                    src = {ln: self.vf[ln][t[2]] for ln in self.lanes}
                    val = {ln: (src[(ln & ~1) | t[4][ln & 1]] + self.vf[ln][t[3]]) & 0xffffffff
                           for ln in self.lanes}
                    for ln in self.lanes:
                        self.vf[ln][t[1]] = val[ln]
                    nxt = None
                else:
                    for ln in self.lanes:
                        self.lane, self.v, self.a = ln, self.vf[ln], self.af[ln]
                        nxt = self.step(t)
            else:
                nxt = self.step(t)
            if nxt == "end":
                return
            pc = self.labels[nxt] if nxt is not None else pc + 1

    LOFF = 16     # v16 = tid * 8 (emit.LOFF)

    def run_wave(self, pc):
        """a wave_begin .. wave_end region (straight-line code, e.g. a copy in
        which every lane of the wave loads for other lanes): run for all 64
        lanes, the lanes outside the simulated ones starting from a copy of the
        first simulated lane's registers with their own tid; returns the pc
        after the region"""
        code = self.code
        end = next(k for k in range(pc, len(code)) if code[k][0] == "wave_end")
        main = self.lanes[0]
        files = {}
        for ln in range(64):
            if ln in self.vf:
                files[ln] = (self.vf[ln], self.af[ln])
            else:
                v = list(self.vf[main])
                v[self.LOFF] = 8 * ln
                files[ln] = (v, list(self.af[main]))
        for k in range(pc + 1, end):
            t = code[k]
            self.pc = k
            m = t[0]
            self.count += 1
            self.hist[m] = self.hist.get(m, 0) + 1
            self.ws += (t[1] + 1) if m == "s_nop" else 1
            if m.startswith("global_"):
                self.seq["vm"] += 1
            if m.startswith("v_") or m.startswith("global_"):
                for ln in range(64):
                    self.lane, (self.v, self.a) = ln, files[ln]
                    self.step(t)
            else:
                self.step(t)
        self.lane, self.v, self.a = main, self.vf[main], self.af[main]
        return end + 1

    def step(self, t):
        m = t[0]
        a = t[1:]
        rd, rd64, wr, wr64 = self.rd, self.rd64, self.wr, self.wr64
        if m == "v_mad_u64_u32":
            r = rd(a[1]) * rd(a[2]) + rd64(a[3])
            wr64(a[0], r)
            self.set_vcc(r >> 64)
        elif m == "v_mad_i64_i32":
            r = sx32(rd(a[1])) * sx32(rd(a[2])) + sx64(rd64(a[3]))
            wr64(a[0], r)
        elif m == "v_mul_lo_u32":
            wr(a[0], rd(a[1]) * rd(a[2]))
        elif m == "v_and_b32":
            wr(a[0], rd(a[1]) & rd(a[2]))
        elif m == "v_or_b32":
            wr(a[0], rd(a[1]) | rd(a[2]))
        elif m == "v_add_u32":
            wr(a[0], rd(a[1]) + rd(a[2]))
        elif m == "v_sub_u32":
            wr(a[0], rd(a[1]) - rd(a[2]))
        elif m == "v_add3_u32":
            wr(a[0], rd(a[1]) + rd(a[2]) + rd(a[3]))
        elif m == "v_sad_u32":   # |s0 - s1| + s2; the emitter relies on s0 >= s1
            x, y = rd(a[1]), rd(a[2])
            assert x >= y, "v_sad_u32: subtraction constant below the subtrahend limb"
            wr(a[0], x - y + rd(a[3]))
        elif m == "v_subrev_u32":
            wr(a[0], rd(a[2]) - rd(a[1]))
        elif m == "v_lshrrev_b32":
            wr(a[0], rd(a[2]) >> (rd(a[1]) & 31))
        elif m == "v_lshlrev_b32":
            wr(a[0], rd(a[2]) << (rd(a[1]) & 31))
        elif m == "v_ashrrev_i32":
            wr(a[0], sx32(rd(a[2])) >> (rd(a[1]) & 31))
        elif m == "v_lshrrev_b64":
            wr64(a[0], rd64(a[2]) >> (rd(a[1]) & 63))
        elif m == "v_ashrrev_i64":
            wr64(a[0], sx64(rd64(a[2])) >> (rd(a[1]) & 63))
        elif m == "v_lshl_add_u64":
            wr64(a[0], (rd64(a[1]) << (rd(a[2]) & 63)) + rd64(a[3]))
        elif m == "v_lshl_add_u32":
            wr(a[0], (rd(a[1]) << (rd(a[2]) & 31)) + rd(a[3]))
        elif m == "v_lshl_or_b32":
            wr(a[0], (rd(a[1]) << (rd(a[2]) & 31)) | rd(a[3]))
        elif m == "v_alignbit_b32":
            wr(a[0], ((rd(a[1]) << 32) | rd(a[2])) >> (rd(a[3]) & 31))
        elif m == "v_bfi_b32":
            msk = rd(a[1])
            wr(a[0], (msk & rd(a[2])) | (~msk & rd(a[3])))
        elif m == "v_cndmask_b32":
            wr(a[0], rd(a[2]) if self.vcc() else rd(a[1]))
        elif m == "v_cndmask_b32_e64":
            msk = rd64(a[3])
            wr(a[0], rd(a[2]) if (msk >> (self.lane % 64)) & 1 else rd(a[1]))
        elif m == "v_mul_u32_u24":
            wr(a[0], (rd(a[1]) & 0xffffff) * (rd(a[2]) & 0xffffff))
        elif m == "v_mov_b32" or m == "v_accvgpr_write_b32" or m == "v_accvgpr_read_b32":
            wr(a[0], rd(a[1]))
        elif m == "v_mov_b64":
            wr64(a[0], rd64(a[1]))
        elif m == "v_cmp_eq_u32_e64":
            self.set_mask(a[0], rd(a[1]) == rd(a[2]))
        elif m == "v_cmp_ne_u32_e64":
            self.set_mask(a[0], rd(a[1]) != rd(a[2]))
        elif m == "v_cmp_lt_u64_e64":
            self.set_mask(a[0], rd64(a[1]) < rd64(a[2]))
        elif m == "s_and_b64":
            wr64(a[0], rd64(a[1]) & rd64(a[2]))
        elif m == "s_or_b64":
            wr64(a[0], rd64(a[1]) | rd64(a[2]))
        elif m == "v_sub_co_u32":
            r = rd(a[1]) - rd(a[2])
            wr(a[0], r)
            self.set_vcc(r < 0)
        elif m == "v_subb_co_u32":
            r = rd(a[1]) - rd(a[2]) - self.vcc()
            wr(a[0], r)
            self.set_vcc(r < 0)
        elif m == "v_xad_u32":
            wr(a[0], (rd(a[1]) ^ rd(a[2])) + rd(a[3]))
        elif m == "v_xor_b32":
            wr(a[0], rd(a[1]) ^ rd(a[2]))
        elif m == "v_or3_b32":
            wr(a[0], rd(a[1]) | rd(a[2]) | rd(a[3]))
        elif m == "v_ffbh_u32":
            x = rd(a[1])
            wr(a[0], 32 - x.bit_length() if x else M32)
        elif m == "v_max_u32":
            wr(a[0], max(rd(a[1]), rd(a[2])))
        elif m == "v_mad_u32_u24":
            wr(a[0], (rd(a[1]) & 0xffffff) * (rd(a[2]) & 0xffffff) + rd(a[3]))
        elif m == "v_cmp_gt_u32":
            self.set_vcc(rd(a[0]) > rd(a[1]))
        elif m == "v_cmp_eq_u32":
            self.set_vcc(rd(a[0]) == rd(a[1]))
        elif m == "v_cmp_ne_u32":
            self.set_vcc(rd(a[0]) != rd(a[1]))
        elif m == "ds_write_b64":
            addr = rd(a[0]) + a[2]
            self.lds[addr] = rd(a[1])
            self.lds[addr + 4] = rd(a[1] + 1)
        elif m == "ds_read_b64":
            addr = rd(a[1]) + a[2]
            if addr in self.lds_dma or addr + 4 in self.lds_dma:
                raise AssertionError("LDS read of 0x%x before its global_load_lds was waited for (instr %d)" % (
                    addr, self.count))
            self.async_wr("lgkm", a[0], self.lds.get(addr, 0))
            self.async_wr("lgkm", a[0] + 1, self.lds.get(addr + 4, 0))
        elif m == "global_load_dwordx2":
            addr = rd64(a[1]) + a[2]
            wr(a[0], self.ld32(addr))
            wr(a[0] + 1, self.ld32(addr + 4))
        elif m == "global_load_lds_dwordx4":
            # 16 bytes from this lane's address into LDS at M0 + 16 lane, landing
            # at a vmcnt wait (the instruction offset is always 0 here)
            addr = rd64(a[0])
            for w in range(4):
                self.lds_dma[self.m0 + 16 * (self.lane % 64) + 4 * w] = (self.seq["vm"], self.ld32(addr + 4 * w))
        elif m == "global_load_dword":
            wr(a[0], self.ld32(rd64(a[1]) + a[2]))
        elif m == "global_store_dwordx2":
            addr = rd64(a[0]) + a[2]
            self.st32(addr, rd(a[1]))
            self.st32(addr + 4, rd(a[1] + 1))
        elif m == "global_store_byte":
            addr = rd64(a[0]) + a[2]
            base = addr & ~3
            sh = 8 * (addr & 3)
            w = self.ld32(base)
            self.st32(base, (w & ~(0xff << sh)) | ((rd(a[1]) & 0xff) << sh))
        elif m == "global_store_dwordx2_s":
            addr = rd64(a[2]) + rd(a[0]) + a[3]
            self.st32(addr, rd(a[1]))
            self.st32(addr + 4, rd(a[1] + 1))
            self.st_inflight[addr] = self.st_inflight[addr + 4] = self.seq["vm"]
        elif m == "global_load_dwordx2_s":
            addr = rd64(a[2]) + rd(a[1]) + a[3]
            if addr in self.st_inflight or addr + 4 in self.st_inflight:
                raise AssertionError("workspace load of 0x%x before its store was waited for (instr %d)" % (
                    addr, self.count))
            self.async_wr("vm", a[0], self.ld32(addr))
            self.async_wr("vm", a[0] + 1, self.ld32(addr + 4))
        elif m == "s_load_dwordx2":
            addr = rd64(a[1]) + a[2]
            wr(a[0], self.ld32(addr))
            wr(a[0] + 1, self.ld32(addr + 4))
        elif m == "s_mov_b32":
            wr(a[0], rd(a[1]))
        elif m in ("s_or_saveexec_b64", "s_mov_b64_exec"):
            pass          # exec: the simulator runs the lanes it is given
        elif m == "v_min_u32":
            wr(a[0], min(rd(a[1]), rd(a[2])))
        elif m == "s_mov_m0":
            self.m0 = rd(a[0])
        elif m == "s_min_u32":
            wr(a[0], min(rd(a[1]), rd(a[2])))
        elif m == "s_mov_b64":
            wr64(a[0], rd64(a[1]))
        elif m == "s_add_u32":
            r = rd(a[1]) + rd(a[2])
            wr(a[0], r)
            self.scc = r >> 32
        elif m == "s_addc_u32":
            r = rd(a[1]) + rd(a[2]) + self.scc
            wr(a[0], r)
            self.scc = r >> 32
        elif m == "s_sub_u32":
            r = rd(a[1]) - rd(a[2])
            wr(a[0], r)
            self.scc = int(r < 0)
        elif m == "s_and_b32":
            r = rd(a[1]) & rd(a[2])
            wr(a[0], r)
            self.scc = int(r != 0)
        elif m == "s_cmp_eq_u32":
            self.scc = int(rd(a[0]) == rd(a[1]))
        elif m == "s_setprio":
            pass
        elif m == "s_cmp_ge_i32":
            self.scc = int(sx32(rd(a[0])) >= sx32(rd(a[1])))
        elif m == "s_cmp_eq_u64":
            self.scc = int(rd64(a[0]) == rd64(a[1]))
        elif m == "s_bitcmp1_b64":
            self.scc = (rd64(a[0]) >> (rd(a[1]) & 63)) & 1
        elif m == "s_mul_i32":
            wr(a[0], rd(a[1]) * rd(a[2]))
        elif m == "s_lshl_b32":
            wr(a[0], rd(a[1]) << (rd(a[2]) & 31))
        elif m == "s_mul_hi_u32":
            wr(a[0], (rd(a[1]) * rd(a[2])) >> 32)
        elif m == "s_and_saveexec_b64":
            if not all(self.vcc_of(ln) for ln in self.lanes):
                return "end"
        elif m == "mark":
            if self.trace is not None:
                if self.lane == self.lanes[0]:
                    while True:
                        vid, limbs, op = next(self.trace)
                        if vid == a[0]:
                            break
                    self.cur_mark = (limbs, op)
                limbs, op = self.cur_mark
                if len(self.lanes) == 2:
                    limbs = limbs[self.lanes.index(self.lane)]
                got = tuple(self.v[a[1] + i] for i in range(14))
                if got != tuple(x & 0xffffffff for x in limbs):   # signed limbs (pdiff) as u32
                    raise AssertionError("first divergence at %r (instr %d): got %s want %s" % (
                        op, self.count, got, tuple(limbs)))
        elif m == "s_waitcnt_lgkm0":
            self.complete("lgkm")
        elif m == "s_waitcnt_vm0":
            self.complete("vm")
        elif m == "s_waitcnt_lgkm":
            self.complete("lgkm", a[0])
        elif m == "s_waitcnt_vm":
            self.complete("vm", a[0])
        elif m in ("s_nop", "label"):
            pass
        elif m == "long_cbranch_scc1":
            return a[0] if self.scc else None
        elif m == "long_cbranch_scc0":
            return None if self.scc else a[0]
        elif m == "long_cbranch_execz":
            return None
        elif m == "s_endpgm":
            return "end"
        else:
            raise NotImplementedError(m)
        return None


def run_lane(code, args, buffers, lane=0, max_steps=10 ** 9, trace=None, pair=False, lds=None):
    """args: 5 u64 kernel arguments; buffers: {base_address: list of u64};
    pair: simulate lanes (lane & ~1, lane | 1) together; lds: {byte address:
    u32} the wave's other lanes write (a table the whole wave stages)"""
    sm = Sim(code, lane, [lane & ~1, lane | 1] if pair else None)
    sm.lds.update(lds or {})
    sm.trace = iter(trace) if trace is not None else None
    for base, words in buffers.items():
        for i, w in enumerate(words):
            sm.mem[base + 8 * i] = w & M32
            sm.mem[base + 8 * i + 4] = (w >> 32) & M32
    karg = 0x1000
    for i, x in enumerate(args):
        sm.mem[karg + 8 * i] = x & M32
        sm.mem[karg + 8 * i + 4] = x >> 32
    sm.s[0], sm.s[1] = karg, 0
    sm.s[2] = lane // 64
    for ln in sm.lanes:
        sm.vf[ln][0] = ln % 64
    sm.run(max_steps)
    return sm
