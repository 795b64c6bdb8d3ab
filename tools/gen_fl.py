#!/usr/bin/env python3
"""Generate pairing_amd/csrc/fl_gen.h: the redundant-limb Montgomery core.

Representation "Fl" (lazy Fq): 14 limbs of nominally 28 bits in 32-bit
registers, value = sum w[i] 2^(28 i), Montgomery radix R = 2^392.  A value
carries a bound u (tracked by the code that uses it):

    every limb <= u (2^28 - 1)    and    value < u * 2q.

A Montgomery product returns u = 1 (limbs < 2^28, value < 2q).  Additions are
limb-wise with no carries (u adds up); a subtraction adds a multiple of q
written with limbs large enough that no limb goes negative (SUB_C below).

Why: on gfx950 a `v_mad_u64_u32` accumulator chain costs the same as
independent mads (measured, profiles/r01_valu_rates2.txt), while every
SGPR-carry op costs more than a mad.  With 28-bit limbs a whole Montgomery
product column (up to 14 a*b and 14 m*q terms, u_a*u_b <= 17) fits in one
64-bit accumulator, so the product is 392 mads + one shift per column and
no carry instructions; additions are 14 plain adds.

The products are leaf subroutines with a fixed register convention, called
with `s_swappc_b64` from inline asm (operands pinned with physical-register
constraints), so every call site costs only the moves into v0..: the tower
code above inlines without duplicating 400-instruction bodies and without
stack traffic.

  pa_fl_sop1   out = a*b / R                v[0:14) a, v[14:28) b -> v[28:42)
  pa_fl_sop2   out = (a*b + c*d) / R        v[0:56)              -> v[56:70)
  pa_fl_sqr    out = a*a / R                v[0:14)              -> v[28:42)
All: out < 2q, limbs < 2^28 (u = 1) given the input bounds checked by the
callers (sum of u_x*u_y over the products <= 17; sqr needs u_a <= 3).
reference: Fq::mul_assign / square / mont_reduce, fq.rs:909-1122 (the same
field value; the limb radix is internal, conversions in fl.h).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_consts import Q, FROB_FQ2_C1, FROB_FQ6_C1, FROB_FQ6_C2, FROB_FQ12_C1  # noqa: E402

NL = 14
LB = 28
MASK = (1 << LB) - 1
RL = 1 << (NL * LB)  # 2^392
QINV = (-pow(Q, -1, 1 << LB)) % (1 << LB)
U_MAX_SUB = 14  # SUB_C tables for subtrahend bounds 1..U_MAX_SUB

# floor(2^400 / q): with T = x13 2^28 + x12 (< 2^50), k = (T KQ) >> 64 is
# floor(V / q) or one less for any V < 2^388 with limbs < 2^32 (checked in
# tests/test_fl_model.py), so V - k q lies in [0, 2q).
KQ = (1 << 400) // Q
assert KQ < (1 << 32)

QS = 40  # q limbs in s[40:53] (low: keeps the hipcc kernels under 80 SGPRs, 8 waves/SIMD)
QI = 54  # qinv in s54



def _write_if_changed(path, text):
    """rewrite a generated header only when its text changes, so that a build
    after an unchanged generator run rebuilds nothing (make compares mtimes)"""
    import os as _os
    if _os.path.exists(path):
        with open(path) as f:
            if f.read() == text:
                return
    with open(path, "w") as f:
        f.write(text)

def limbs(v, n=NL):
    return [(v >> (LB * i)) & MASK for i in range(n)]


def sub_constant(ub):
    """C = k q with limbs c_i >= ub (2^28-1) (i < 13), c_13 >= ub 2^18 + 1: subtracting
    any value of bound ub limb-wise from a + C never goes negative.  Returns
    (limbs, u_C) with u_C the bound of C itself."""
    lo = [ub * MASK] * (NL - 1) + [ub * (1 << 18)]
    minv = sum(c << (LB * i) for i, c in enumerate(lo))
    k = -(-minv // Q)
    d = k * Q - minv
    c = [lo[i] + ((d >> (LB * i)) & MASK) for i in range(NL - 1)]
    c.append(lo[NL - 1] + (d >> (LB * (NL - 1))))
    assert sum(x << (LB * i) for i, x in enumerate(c)) == k * Q
    assert all(x < (1 << 32) for x in c)
    ulimb = max(-(-x // MASK) for x in c)
    uval = -(-(k * Q) // (2 * Q))
    return c, max(ulimb, uval)


def sub_constant2(ulimb, vtop):
    """C = k q with limbs c_i >= ulimb (2^28-1) (i < 13) and c_13 >= vtop 2^18 + 1:
    for a subtrahend of limb bound ulimb and value bound vtop 2q (its top limb is
    below value / 2^364 < vtop 2^18).  Returns (limbs, limb bound of C, value
    bound of C in units of 2q)."""
    lo = [ulimb * MASK] * (NL - 1) + [vtop * (1 << 18)]
    minv = sum(c << (LB * i) for i, c in enumerate(lo))
    k = -(-minv // Q)
    d = k * Q - minv
    c = [lo[i] + ((d >> (LB * i)) & MASK) for i in range(NL - 1)]
    c.append(lo[NL - 1] + (d >> (LB * (NL - 1))))
    assert sum(x << (LB * i) for i, x in enumerate(c)) == k * Q
    assert all(x < (1 << 32) for x in c)
    return c, max(-(-x // MASK) for x in c), (k * Q) // (2 * Q) + 1   # value < that 2q, strictly


def leaf_sop(K):
    A = lambda p, i: 28 * p + i
    B = lambda p, i: 28 * p + 14 + i
    OUT = 28 * K
    ACC = OUT + 14
    M = ACC + 2
    acc = "v[%d:%d]" % (ACC, ACC + 1)
    L = []
    L.append(".p2align 8")
    L.append("pa_fl_sop%d:" % K)
    for i, w in enumerate(limbs(Q)):
        L.append("s_mov_b32 s%d, 0x%x" % (QS + i, w))
    L.append("s_mov_b32 s%d, 0x%x" % (QI, QINV))
    first = True
    for k in range(2 * NL - 1):
        for p in range(K):
            for i in range(max(0, k - (NL - 1)), min(k, NL - 1) + 1):
                L.append("v_mad_u64_u32 %s, vcc, v%d, v%d, %s" % (acc, A(p, i), B(p, k - i), "0" if first else acc))
                first = False
        for i in range(max(0, k - (NL - 1)), min(k - 1, NL - 1) + 1):
            L.append("v_mad_u64_u32 %s, vcc, v%d, s%d, %s" % (acc, M + i, QS + k - i, acc))
        if k < NL:
            L.append("v_mul_lo_u32 v%d, v%d, s%d" % (M + k, ACC, QI))
            L.append("v_and_b32 v%d, 0x%x, v%d" % (M + k, MASK, M + k))
            L.append("v_mad_u64_u32 %s, vcc, v%d, s%d, %s" % (acc, M + k, QS, acc))
        else:
            L.append("v_and_b32 v%d, 0x%x, v%d" % (OUT + k - NL, MASK, ACC))
        L.append("v_lshrrev_b64 %s, %d, %s" % (acc, LB, acc))
    L.append("v_mov_b32 v%d, v%d" % (OUT + NL - 1, ACC))
    L.append("s_setpc_b64 s[30:31]")
    return L, OUT, list(range(ACC, M + NL))


def leaf_sqr():
    A = lambda i: i
    A2 = lambda i: 14 + i
    OUT, ACC = 28, 42
    M = 44
    acc = "v[%d:%d]" % (ACC, ACC + 1)
    L = [".p2align 8", "pa_fl_sqr:"]
    for i in range(NL):
        L.append("v_lshlrev_b32 v%d, 1, v%d" % (A2(i), A(i)))
    for i, w in enumerate(limbs(Q)):
        L.append("s_mov_b32 s%d, 0x%x" % (QS + i, w))
    L.append("s_mov_b32 s%d, 0x%x" % (QI, QINV))
    first = True
    for k in range(2 * NL - 1):
        for i in range(max(0, k - (NL - 1)), min(k, NL - 1) + 1):
            j = k - i
            if i < j:
                L.append("v_mad_u64_u32 %s, vcc, v%d, v%d, %s" % (acc, A(i), A2(j), "0" if first else acc))
            elif i == j:
                L.append("v_mad_u64_u32 %s, vcc, v%d, v%d, %s" % (acc, A(i), A(i), "0" if first else acc))
            else:
                continue
            first = False
        for i in range(max(0, k - (NL - 1)), min(k - 1, NL - 1) + 1):
            L.append("v_mad_u64_u32 %s, vcc, v%d, s%d, %s" % (acc, M + i, QS + k - i, acc))
        if k < NL:
            L.append("v_mul_lo_u32 v%d, v%d, s%d" % (M + k, ACC, QI))
            L.append("v_and_b32 v%d, 0x%x, v%d" % (M + k, MASK, M + k))
            L.append("v_mad_u64_u32 %s, vcc, v%d, s%d, %s" % (acc, M + k, QS, acc))
        else:
            L.append("v_and_b32 v%d, 0x%x, v%d" % (OUT + k - NL, MASK, ACC))
        L.append("v_lshrrev_b64 %s, %d, %s" % (acc, LB, acc))
    L.append("v_mov_b32 v%d, v%d" % (OUT + NL - 1, ACC))
    L.append("s_setpc_b64 s[30:31]")
    return L, OUT, list(range(14, 28)) + list(range(ACC, M + NL))


CALL = ("s_getpc_b64 s[30:31]\\n\\t"
        "s_add_u32 s30, s30, %s@rel32@lo+4\\n\\t"
        "s_addc_u32 s31, s31, %s@rel32@hi+12\\n\\t"
        "s_swappc_b64 s[30:31], s[30:31]")


def wrapper(name, leaf, nin, out, clob):
    """C++ wrapper: inputs are Fl refs x0..x{nin-1} placed at v[0 : 14 nin)."""
    args = ", ".join("const uint32_t* x%d" % i for i in range(nin))
    L = ["PA_DEV void %s(uint32_t* r, %s) {" % (name, args)]
    L.append("    uint64_t o0, o1, o2, o3, o4, o5, o6;")
    outs = ", ".join('"={v[%d:%d]}"(o%d)' % (out + 2 * j, out + 2 * j + 1, j) for j in range(7))
    ins = []
    for x in range(nin):
        for j in range(7):
            base = 14 * x + 2 * j
            ins.append('"{v[%d:%d]}"(fl_pair(x%d, %d))' % (base, base + 1, x, j))
    clobs = ['"v%d"' % c for c in clob] + ['"s%d"' % s for s in [30, 31] + list(range(QS, QS + NL)) + [QI]]
    clobs += ['"vcc"', '"scc"']
    L.append('    asm volatile("%s"' % (CALL % (leaf, leaf)))
    L.append("        : " + outs)
    L.append("        : " + ", ".join(ins))
    L.append("        : " + ", ".join(clobs) + ");")
    for j in range(7):
        L.append("    r[%d] = (uint32_t)o%d; r[%d] = (uint32_t)(o%d >> 32);" % (2 * j, j, 2 * j + 1, j))
    L.append("}")
    return L


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.abspath(__file__)), "..", "pairing_amd", "csrc", "fl_gen.h")
    H = ["// GENERATED by tools/gen_fl.py -- do not edit.", "#pragma once", "#include <stdint.h>", "",
         "namespace pa {", ""]
    H.append("constexpr int FL_NL = %d;" % NL)
    H.append("constexpr uint32_t FL_MASK = 0x%xu;" % MASK)
    H.append("__constant__ const uint32_t FL_Q[%d] = {%s};" % (NL, ", ".join("0x%xu" % w for w in limbs(Q))))
    # conversion constants (canonical, u = 1): into Fl from R=2^384 words, back out
    H.append("// to_fl: mont(x_384, 2^400 mod q) = x 2^392;  from_fl: mont(y, 2^384 mod q) = x 2^384")
    H.append("__constant__ const uint32_t FL_TO[%d] = {%s};" % (
        NL, ", ".join("0x%xu" % w for w in limbs(pow(2, 400, Q)))))
    H.append("__constant__ const uint32_t FL_FROM[%d] = {%s};" % (
        NL, ", ".join("0x%xu" % w for w in limbs(pow(2, 384, Q)))))
    mt = lambda v: limbs(v * RL % Q)
    arr = lambda v: "{%s}" % ", ".join("0x%xu" % w for w in mt(v))
    H.append("__constant__ const uint32_t FL_ONE[%d] = %s;" % (NL, arr(1)))
    H.append("// red(): quotient estimate k = (T * FL_KQ) >> 64, T = top two limbs (x13 2^28 + x12)")
    H.append("constexpr uint32_t FL_KQ = 0x%xu;" % KQ)
    H.append("// Montgomery digit factor -q^-1 mod 2^28 (the leaves' s%d; coop_quad.h)" % QI)
    H.append("constexpr uint32_t FL_QINV = 0x%xu;" % QINV)
    H.append("__constant__ const uint32_t FL_FROB_FQ2_C1[2][%d] = {%s};" % (NL, ", ".join(arr(v) for v in FROB_FQ2_C1)))
    for nm, tab in (("FROB_FQ6_C1", FROB_FQ6_C1), ("FROB_FQ6_C2", FROB_FQ6_C2), ("FROB_FQ12_C1", FROB_FQ12_C1)):
        H.append("__constant__ const uint32_t FL_%s[%d][2][%d] = {\n    %s};" % (
            nm, len(tab), NL, ",\n    ".join("{%s, %s}" % (arr(c0), arr(c1)) for c0, c1 in tab)))
    H.append("// SUB_C[u-1]: k q with limbs >= u (2^28-1); SUB_CU[u-1]: its own bound")
    rows, us = [], []
    for ub in range(1, U_MAX_SUB + 1):
        c, uc = sub_constant(ub)
        rows.append("{%s}" % ", ".join("0x%xu" % w for w in c))
        us.append(str(uc))
    H.append("__constant__ const uint32_t FL_SUB_C[%d][%d] = {\n    %s};" % (U_MAX_SUB, NL, ",\n    ".join(rows)))
    H.append("constexpr int FL_SUB_CU[%d] = {%s};" % (U_MAX_SUB, ", ".join(us)))
    H.append("")
    # leaves
    # hipcc drops file-scope asm from the device compilation, so the leaves live
    # in a never-launched holder kernel that starts with s_endpgm
    H.append("namespace {")
    H.append("__global__ __attribute__((used)) void pa_fl_leaf_holder() {")
    H.append("asm volatile(R\"PAFL(")
    H.append("s_endpgm")
    leaves = []
    for K in (1, 2):
        body, out, clob = leaf_sop(K)
        leaves.append(("pa_fl_sop%d" % K, body, out, clob, 2 * K))
    body, out, clob = leaf_sqr()
    leaves.append(("pa_fl_sqr", body, out, clob, 1))
    for name, body, *_ in leaves:
        H.extend(body)
    H.append(")PAFL\");")
    H.append("}")
    H.append("}  // namespace")
    H.append("")
    H.append("PA_DEV uint64_t fl_pair(const uint32_t* x, int j) {")
    H.append("    return (uint64_t)x[2 * j] | ((uint64_t)x[2 * j + 1] << 32);")
    H.append("}")
    for name, body, out, clob, nin in leaves:
        cname = {"pa_fl_sop1": "fl_mul_leaf", "pa_fl_sop2": "fl_sop2_leaf", "pa_fl_sqr": "fl_sqr_leaf"}[name]
        H.extend(wrapper(cname, name, nin, out, clob))
        H.append("")
    H.append("}  // namespace pa")
    _write_if_changed(out_path, "\n".join(H) + "\n")
    n_instr = {name: sum(1 for l in body if l and not l.endswith(":") and not l.startswith(".")) for name, body, *_ in leaves}
    print("wrote %s: %s" % (out_path, n_instr))


if __name__ == "__main__":
    main()
