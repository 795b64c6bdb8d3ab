"""Render emitted instruction tuples (emit.py) as gfx950 assembly with an
amdhsa kernel descriptor + code-object metadata, and assemble / link it
into a code object (.hsaco) with the ROCm LLVM tools."""
import os

TWO_WAVES = os.environ.get("PGEN_TWO_WAVES", "0") == "1"   # see emit.py
import subprocess

LLVM = "/opt/rocm/lib/llvm/bin"

W64 = {  # operand positions that are 64-bit register pairs, per mnemonic
    "v_mad_u64_u32": (0, 3), "v_mad_i64_i32": (0, 3), "v_mov_b64": (0, 1),
    "v_lshrrev_b64": (0, 2), "v_ashrrev_i64": (0, 2), "v_lshl_add_u64": (0, 1, 3),
    "ds_write_b64": (1,), "ds_read_b64": (0,),
    "global_load_dwordx2": (0, 1), "global_load_dword": (1,), "global_store_dwordx2": (0, 1),
    "global_store_byte": (0,), "global_load_lds_dwordx4": (0,), "global_store_dwordx2_s": (1, 2), "global_load_dwordx2_s": (0, 2),
    "s_load_dwordx2": (0, 1), "s_mov_b64": (0, 1), "s_and_saveexec_b64": (0,), "s_bitcmp1_b64": (0,),
    "s_cmp_eq_u64": (0,), "v_cmp_eq_u32_e64": (0,), "v_cmp_ne_u32_e64": (0,),
    "v_cmp_lt_u64_e64": (0, 1, 2), "s_and_b64": (0, 1, 2), "s_or_b64": (0, 1, 2),
}


OFFSET_LAST = {"ds_write_b64", "ds_read_b64", "global_load_dwordx2", "global_load_dword", "global_store_dwordx2",
               "global_store_byte", "global_store_dwordx2_s", "global_load_dwordx2_s", "s_load_dwordx2"}


def reg(x, wide=False):
    if isinstance(x, tuple):
        v = x[1]
        return str(v) if -16 <= v <= 64 else "0x%x" % (v & 0xffffffff)
    if x >= 512:
        n = x - 512
        if n == 106:
            return "vcc"
        return "s[%d:%d]" % (n, n + 1) if wide else "s%d" % n
    if x >= 256:
        n = x - 256
        return "a[%d:%d]" % (n, n + 1) if wide else "a%d" % n
    return "v[%d:%d]" % (x, x + 1) if wide else "v%d" % x


class Renderer:
    def __init__(self, code):
        self.code = code
        self.n = 0
        self.defined = set()

    def ops(self, m, args):
        w = W64.get(m, ())
        return [reg(a, i in w) for i, a in enumerate(args)]

    def jump(self, target, cond_skip):
        """cond_skip: the short branch that skips the long jump (or None)"""
        self.n += 1
        nb, pc = ".Lnb_%d" % self.n, ".Lpc_%d" % self.n
        back = target in self.defined
        out = []
        if cond_skip:
            out.append("%s %s" % (cond_skip, nb))
        out += ["s_getpc_b64 s[30:31]", "%s:" % pc,
                "s_add_u32 s30, s30, %s-%s" % (target, pc),
                "s_addc_u32 s31, s31, %s" % ("-1" if back else "0"),
                "s_setpc_b64 s[30:31]"]
        if cond_skip:
            out.append("%s:" % nb)
        return out

    def line(self, t):
        m, a = t[0], t[1:]
        if m in ("label", "long_cbranch_scc1", "long_cbranch_scc0", "long_cbranch_execz"):
            o = None
        else:
            o = self.ops(m, [x if not (isinstance(x, int) and m in OFFSET_LAST and i == len(a) - 1) else ("k", x)
                             for i, x in enumerate(a)])
        if m == "label":
            self.defined.add(a[0])
            return ["%s:" % a[0]]
        if m == "long_cbranch_scc1":
            return self.jump(a[0], "s_cbranch_scc0")
        if m == "long_cbranch_scc0":
            return self.jump(a[0], "s_cbranch_scc1")
        if m == "long_cbranch_execz":
            return self.jump(a[0], "s_cbranch_execnz")
        if m in ("v_mad_u64_u32", "v_mad_i64_i32"):
            return ["%s %s, vcc, %s, %s, %s" % (m, o[0], o[1], o[2], o[3])]
        if m.startswith("v_cmp_") and m.endswith("_e64"):
            return ["%s %s, %s, %s" % (m, o[0], o[1], o[2])]
        if m.startswith("v_cmp_"):
            return ["%s vcc, %s, %s" % (m, o[0], o[1])]
        if m == "v_sub_co_u32":
            return ["v_sub_co_u32_e32 %s, vcc, %s, %s" % (o[0], o[1], o[2])]
        if m == "v_subb_co_u32":
            return ["v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (o[0], o[1], o[2])]
        if m == "v_cndmask_b32":
            return ["v_cndmask_b32 %s, %s, %s, vcc" % (o[0], o[1], o[2])]
        if m == "v_cndmask_b32_e64":
            return ["v_cndmask_b32_e64 %s, %s, %s, %s" % (o[0], o[1], o[2], reg(a[3], True))]
        if m == "v_add_u32_dpp":
            q = a[3]
            return ["v_add_u32_dpp %s, %s, %s quad_perm:[%d,%d,%d,%d] row_mask:0xf bank_mask:0xf" % (
                o[0], o[1], o[2], q[0], q[1], q[0] + 2, q[1] + 2)]
        if m == "v_mov_b32_dpp_swap":
            return ["v_mov_b32_dpp %s, %s quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" % (o[0], o[1])]
        if m == "v_mov_b32_dpp_bcast":
            r = a[2]
            return ["v_mov_b32_dpp %s, %s quad_perm:[%d,%d,%d,%d] row_mask:0xf bank_mask:0xf" % (
                o[0], o[1], r, r, r + 2, r + 2)]
        if m == "v_sub_u32_dpp_bcast0":
            return ["v_sub_u32_dpp %s, %s, %s quad_perm:[0,0,2,2] row_mask:0xf bank_mask:0xf" % (o[0], o[1], o[2])]
        if m == "v_cndmask_b32_dpp_swap":
            return ["v_cndmask_b32_dpp %s, %s, %s, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" % (
                o[0], o[1], o[2])]
        if m == "ds_write_b64":
            return ["ds_write_b64 %s, %s offset:%d" % (o[0], o[1], a[2])]
        if m == "ds_read_b64":
            return ["ds_read_b64 %s, %s offset:%d" % (o[0], o[1], a[2])]
        if m in ("global_load_dwordx2", "global_load_dword"):
            return ["%s %s, %s, off offset:%d" % (m, o[0], o[1], a[2])]
        if m == "global_store_dwordx2":
            return ["global_store_dwordx2 %s, %s, off offset:%d" % (o[0], o[1], a[2])]
        if m == "global_store_byte":
            return ["global_store_byte %s, %s, off offset:%d" % (o[0], o[1], a[2])]
        if m == "global_store_dwordx2_s":
            return ["global_store_dwordx2 %s, %s, %s offset:%d" % (o[0], o[1], o[2], a[3])]
        if m == "global_load_dwordx2_s":
            return ["global_load_dwordx2 %s, %s, %s offset:%d" % (o[0], o[1], o[2], a[3])]
        if m in ("wave_begin", "wave_end"):
            return []
        if m == "s_or_saveexec_b64":
            return ["s_or_saveexec_b64 %s, %s" % (reg(a[0], True), o[1])]
        if m == "s_mov_b64_exec":
            return ["s_mov_b64 exec, %s" % reg(a[0], True)]
        if m == "s_mov_m0":
            return ["s_mov_b32 m0, %s" % o[0]]
        if m == "global_load_lds_dwordx4":
            return ["global_load_lds_dwordx4 %s, off" % o[0]]
        if m == "s_load_dwordx2":
            return ["s_load_dwordx2 %s, %s, 0x%x" % (o[0], o[1], a[2])]
        if m == "s_waitcnt_lgkm0":
            return ["s_waitcnt lgkmcnt(0)"]
        if m == "s_waitcnt_vm0":
            return ["s_waitcnt vmcnt(0)"]
        if m == "s_waitcnt_vm":
            return ["s_waitcnt vmcnt(%d)" % a[0]]
        if m == "s_waitcnt_lgkm":
            return ["s_waitcnt lgkmcnt(%d)" % a[0]]
        if m == "s_setprio":
            return ["s_setprio %d" % a[0]]
        if m == "s_nop":
            return ["s_nop %d" % a[0]]
        if m == "s_and_saveexec_b64":
            return ["s_and_saveexec_b64 %s, vcc" % o[0]]
        if m == "s_endpgm":
            return ["s_endpgm"]
        return ["%s %s" % (m, ", ".join(o))]

    def text(self):
        out = []
        for t in self.code:
            out.extend(self.line(t))
        return out


def kernel_asm(name, code, lds_bytes, nargs=5, lanes=1, nvgpr=256, mem_slots=None, nsgpr=96):
    """mem_slots: the HBM spill slots per wave the code uses, exported as the
    global `<name>_mem_slots` so the loader (gen_launch.hip) can refuse a code
    object that needs a larger workspace than the library allocates"""
    body = Renderer(code).text()
    args = "\n".join(
        "      - .offset: %d\n        .size: 8\n        .value_kind: %s%s" % (
            8 * k, "by_value" if k == 3 else "global_buffer",
            "" if k == 3 else "\n        .address_space: global")
        for k in range(nargs))
    return """\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"
\t.text
\t.globl {name}
\t.p2align 8
\t.type {name},@function
{name}:
{body}
.Lfunc_end_{name}:
\t.size {name}, .Lfunc_end_{name}-{name}
{memsym}
\t.rodata
\t.p2align 6
\t.amdhsa_kernel {name}
\t\t.amdhsa_group_segment_fixed_size {lds}
\t\t.amdhsa_private_segment_fixed_size 0
\t\t.amdhsa_kernarg_size {kb}
\t\t.amdhsa_user_sgpr_count 2
\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1
\t\t.amdhsa_system_sgpr_workgroup_id_x 1
\t\t.amdhsa_system_vgpr_workitem_id 0
\t\t.amdhsa_next_free_vgpr {nfree}
\t\t.amdhsa_next_free_sgpr {nsgpr}
\t\t.amdhsa_accum_offset {aoff}
\t\t.amdhsa_reserve_vcc 1
\t\t.amdhsa_float_denorm_mode_32 3
\t\t.amdhsa_float_denorm_mode_16_64 3
\t.end_amdhsa_kernel

\t.amdgpu_metadata
---
amdhsa.version: [ 1, 2 ]
amdhsa.kernels:
  - .name: {name}
    .symbol: {name}.kd
    .kernarg_segment_size: {kb}
    .kernarg_segment_align: 8
    .group_segment_fixed_size: {lds}
    .private_segment_fixed_size: 0
    .wavefront_size: 64
    .sgpr_count: {sgpr_count}
    .vgpr_count: {nfree}
    .agpr_count: {nagpr}
    .max_flat_workgroup_size: 64
    .args:
{args}
...
\t.end_amdgpu_metadata
""".format(name=name, body="\n".join(body), lds=lds_bytes, kb=8 * nargs, args=args,
           memsym="" if mem_slots is None else
           "\n\t.rodata\n\t.globl {n}_mem_slots\n\t.p2align 2\n\t.type {n}_mem_slots,@object\n"
           "{n}_mem_slots:\n\t.long {m}\n\t.size {n}_mem_slots, 4\n".format(n=name, m=int(mem_slots)),
           nfree=512 if lanes == 1 and not TWO_WAVES else 256, aoff=nvgpr, nsgpr=nsgpr, sgpr_count=nsgpr + 6,
           nagpr=(512 if lanes == 1 and not TWO_WAVES else 256) - nvgpr)


def assemble(asm_text, out_hsaco, workdir):
    os.makedirs(workdir, exist_ok=True)
    s = os.path.join(workdir, os.path.basename(out_hsaco) + ".s")
    o = os.path.join(workdir, os.path.basename(out_hsaco) + ".o")
    with open(s, "w") as f:
        f.write(asm_text)
    subprocess.run([os.path.join(LLVM, "clang"), "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                    "-mcpu=gfx950", "-c", s, "-o", o], check=True)
    subprocess.run([os.path.join(LLVM, "ld.lld"), "-shared", o, "-o", out_hsaco], check=True)
    return out_hsaco
