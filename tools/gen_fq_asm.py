#!/usr/bin/env python3
"""Generate pairing_amd/csrc/fq_mul_gen.h: hazard-free product-scanning (FIPS)
Montgomery multiplication for gfx950 with the v_mad_u64_u32 carry-out.

Why generated: each 32x32 product is `v_mad_u64_u32 acc, c, x, y, acc`
(carry-out to an SGPR pair) + `v_addc_co_u32 ov, c, 0, ov, c`, 2 VALU
instructions against ~4.5 for the compiler's CIOS lowering.  gfx950 needs
one wait state between a VALU writing a carry SGPR and the VALU reading it
(hipcc pads its own carry chains with `s_nop 0`), so products of N >= 2
independent chains are interleaved round-robin, each chain with its own
carry pair: every carry read is >= 1 instruction after its write.  hipcc
pads one `s_nop 0` after every asm statement, so each statement carries
up to PER_BLOCK products per chain.  Asm statements stay small (< 40
operands): very large operand lists make the register allocator blow up.

Functions:
  fq_mul_x1(r, a, b)               one product, split into an a*b chain and
                                   an m*q chain merged once per column
  fq_mul_x2(r0,a0,b0, r1,a1,b1)    two independent products
  fq_mul_x3(r0,a0,b0, ..., r2,a2,b2)
All return canonical (< q) Montgomery products, bit-identical to
Fq::mul_assign (fq.rs:909-960).
"""
import os

PER_BLOCK = 4



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

def block(chains, prods):
    """prods: list of (chain, x_expr, y_expr, y_is_sgpr) for one asm statement."""
    text = []
    used = sorted({c for c, *_ in prods})
    # outputs: acc_c (+&v 64), ov_c (+&v), carry_c (=&s 64).  The accumulators
    # are early-clobber: they are written before later inputs are read, and
    # without '&' the compiler may give an input that holds the same value
    # (e.g. a zero word of a constant operand) the accumulator's register.
    out_list = []
    for c in used:
        out_list.append(('"+&v"', "acc%s" % chains[c]))
        out_list.append(('"+&v"', "ov%s" % chains[c]))
    for c in used:
        out_list.append(('"=&s"', "cf%s" % chains[c]))
    in_list = []
    in_index = {}

    def inp(cons, expr):
        k = (cons, expr)
        if k not in in_index:
            in_index[k] = len(out_list) + len(in_list)
            in_list.append(k)
        return in_index[k]

    oidx = {e: i for i, (_, e) in enumerate(out_list)}
    by_chain = {c: [p for p in prods if p[0] == c] for c in used}
    rounds = max(len(v) for v in by_chain.values())
    for r in range(rounds):
        live = [c for c in used if r < len(by_chain[c])]
        for c in live:
            _, x, y, ys = by_chain[c][r]
            xi = inp('"v"', x)
            yi = inp('"s"' if ys else '"v"', y)
            text.append("v_mad_u64_u32 %%%d, %%%d, %%%d, %%%d, %%%d" % (
                oidx["acc%s" % chains[c]], oidx["cf%s" % chains[c]], xi, yi, oidx["acc%s" % chains[c]]))
        if len(live) == 1:
            text.append("s_nop 0")  # lone chain: pad the carry hazard ourselves
        for c in live:
            text.append("v_addc_co_u32 %%%d, %%%d, 0, %%%d, %%%d" % (
                oidx["ov%s" % chains[c]], oidx["cf%s" % chains[c]], oidx["ov%s" % chains[c]],
                oidx["cf%s" % chains[c]]))
    asm = "\\n\\t".join(text)
    outs_s = ", ".join("%s(%s)" % (k, e) for k, e in out_list)
    ins_s = ", ".join("%s(%s)" % (k, e) for k, e in in_list)
    return '    asm("%s"\n        : %s\n        : %s);' % (asm, outs_s, ins_s)


def gen(n_chains, name):
    ids = [str(i) for i in range(n_chains)]
    split = n_chains == 1  # x1: chain "0" = a*b products, chain "B" = m*q products
    chains = ids + (["B"] if split else [])
    args = ", ".join("Fq& r%s, const Fq& a%s, const Fq& b%s" % (i, i, i) for i in ids)
    L = ["PA_DEV void %s(%s) {" % (name, args)]
    for i in ids:
        L.append("    uint32_t m%s[12], t%s[12];" % (i, i))
    for c in chains:
        L.append("    uint64_t acc%s = 0, cf%s;" % (c, c))
        L.append("    uint32_t ov%s = 0;" % c)
    for k in range(23):
        prods = []
        for ci, i in enumerate(ids):
            ab = [(ci, "a%s.w[%d]" % (i, j), "b%s.w[%d]" % (i, k - j), False)
                  for j in range(max(0, k - 11), min(k, 11) + 1)]
            mq = [(ci if not split else 1, "m%s[%d]" % (i, j), "PA_Q%d" % (k - j), True)
                  for j in range(max(0, k - 11), min(k - 1, 11) + 1)]
            prods.append(ab + mq)
        # interleave: emit blocks of PER_BLOCK products per chain
        if split:
            flat = prods[0]
            per = {0: [p for p in flat if p[0] == 0], 1: [p for p in flat if p[0] == 1]}
        else:
            per = {ci: prods[ci] for ci in range(n_chains)}
        nblocks = max((len(v) + PER_BLOCK - 1) // PER_BLOCK for v in per.values())
        for b in range(nblocks):
            bp = []
            for ci, v in per.items():
                bp += v[b * PER_BLOCK:(b + 1) * PER_BLOCK]
            if bp:
                L.append(block(chains, bp))
        if split:
            # merge the m*q accumulator into the a*b accumulator (96-bit add)
            L.append("    { uint64_t s = acc0 + accB; ov0 += ovB + (uint32_t)(s < acc0); acc0 = s; accB = 0; ovB = 0; }")
        if k < 12:
            for i in ids:
                L.append("    m%s[%d] = (uint32_t)acc%s * PA_INV32;" % (i, k, i))
            L.append(block(chains, [(ci, "m%s[%d]" % (i, k), "PA_Q0", True) for ci, i in enumerate(ids)]))
        else:
            for i in ids:
                L.append("    t%s[%d] = (uint32_t)acc%s;" % (i, k - 12, i))
        for i in ids:
            L.append("    acc%s = (acc%s >> 32) | ((uint64_t)ov%s << 32); ov%s = 0;" % (i, i, i, i))
    for i in ids:
        L.append("    t%s[11] = (uint32_t)acc%s;" % (i, i))
        L.append("    fq_reduce_once(r%s, t%s);" % (i, i))
    L.append("}")
    return "\n".join(L)


Q_WORDS = ["0xffffaaab", "0xb9feffff", "0xb153ffff", "0x1eabfffe", "0xf6b0f624", "0x6730d2a0",
           "0xf38512bf", "0x64774b84", "0x434bacd7", "0x4b1ba7b6", "0x397fe69a", "0x1a0111ea"]


def gen_addsub():
    """fq_add / fq_sub: two interleaved 12-word carry chains (one VOP3b with an
    SGPR-pair carry, one VOP2 with the literal q word and VCC), so every carry
    is read two instructions after it is written, then one `s_nop 1` and 12
    v_cndmask.  37 VALU slots against ~150 for hipcc's lowering."""
    # operands: 0..11 = x (=&v), 12..23 = y (=&v), 24 = c (=&s), 25..36 = a, 37..48 = b,
    # 49..60 = q words in VGPRs (a VOP2 carry op reads VCC, so a literal or SGPR
    # second operand would exceed gfx9's one-read constant bus)
    QV = lambda i: "%%%d" % (49 + i)
    A = lambda i: "%%%d" % (25 + i)
    B = lambda i: "%%%d" % (37 + i)
    X = lambda i: "%%%d" % i
    Y = lambda i: "%%%d" % (12 + i)
    C = "%24"
    outs = ", ".join('"=&v"(x[%d])' % i for i in range(12)) + ", " + \
        ", ".join('"=&v"(y[%d])' % i for i in range(12)) + ', "=&s"(c)'
    ins = ", ".join('"v"(a.w[%d])' % i for i in range(12)) + ", " + ", ".join('"v"(b.w[%d])' % i for i in range(12)) \
        + ", " + ", ".join('"v"(PA_Q%d)' % i for i in range(12))

    def body(first_a, next_a, first_b, next_b, select):
        t = []
        for i in range(12):
            t.append((first_a if i == 0 else next_a)(i))
            t.append((first_b if i == 0 else next_b)(i))
        t.append("s_nop 1")
        t += [select(i) for i in range(12)]
        return "\\n\\t".join(t)

    # add: x = a + b (SGPR carry), y = x - q (VCC borrow); keep x iff y borrowed
    add_text = body(lambda i: "v_add_co_u32 %s, %s, %s, %s" % (X(i), C, A(i), B(i)),
                    lambda i: "v_addc_co_u32 %s, %s, %s, %s, %s" % (X(i), C, A(i), B(i), C),
                    lambda i: "v_sub_co_u32 %s, vcc, %s, %s" % (Y(i), X(i), QV(i)),
                    lambda i: "v_subb_co_u32 %s, vcc, %s, %s, vcc" % (Y(i), X(i), QV(i)),
                    lambda i: "v_cndmask_b32 %s, %s, %s, vcc" % (X(i), Y(i), X(i)))
    # sub: x = a - b (SGPR borrow), y = x + q (VCC carry); keep y iff x borrowed
    sub_text = body(lambda i: "v_sub_co_u32 %s, %s, %s, %s" % (X(i), C, A(i), B(i)),
                    lambda i: "v_subb_co_u32 %s, %s, %s, %s, %s" % (X(i), C, A(i), B(i), C),
                    lambda i: "v_add_co_u32 %s, vcc, %s, %s" % (Y(i), X(i), QV(i)),
                    lambda i: "v_addc_co_u32 %s, vcc, %s, %s, vcc" % (Y(i), X(i), QV(i)),
                    lambda i: "v_cndmask_b32_e64 %s, %s, %s, %s" % (X(i), X(i), Y(i), C))
    out = []
    for name, text, ref in (("fq_add", add_text, "fq.rs:812-819: a + b, minus q if >= q"),
                            ("fq_sub", sub_text, "fq.rs:830-838: a - b, plus q on borrow")):
        out.append("// %s" % ref)
        out.append("PA_DEV void %s(Fq& r, const Fq& a, const Fq& b) {" % name)
        out.append("    uint32_t x[12], y[12];")
        out.append("    uint64_t c;")
        out.append('    asm("%s"\n        : %s\n        : %s\n        : "vcc");' % (text, outs, ins))
        out.append("#pragma unroll")
        out.append("    for (int i = 0; i < 12; i++) r.w[i] = x[i];")
        out.append("}")
    out.append("PA_DEV void fq_dbl(Fq& r, const Fq& a) { fq_add(r, a, a); }  // fq.rs:821-828")
    out.append("// fq.rs:840-847: q - a unless a == 0 (0 - a reduces to exactly that)")
    out.append("PA_DEV void fq_neg(Fq& r, const Fq& a) {")
    out.append("    Fq z;")
    out.append("    fq_zero(z);")
    out.append("    fq_sub(r, z, a);")
    out.append("}")
    return "\n".join(out)


def main():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "pairing_amd", "csrc", "fq_mul_gen.h")
    body = [
        "// GENERATED by tools/gen_fq_asm.py -- do not edit.",
        "// Hazard-free FIPS Montgomery multiplication on v_mad_u64_u32 carry-out (see the generator).",
        "#pragma once",
        '#include "fq.h"',
        "namespace pa {",
        gen_addsub(),
        gen(1, "fq_mul_x1"),
        gen(2, "fq_mul_x2"),
        gen(3, "fq_mul_x3"),
        "PA_DEV void fq_mul(Fq& r, const Fq& a, const Fq& b) { fq_mul_x1(r, a, b); }",
        "PA_DEV void fq_sqr(Fq& r, const Fq& a) { fq_mul_x1(r, a, a); }",
        "}  // namespace pa",
        "",
    ]
    _write_if_changed(out, "\n".join(body))
    print("wrote", out)


if __name__ == "__main__":
    main()
