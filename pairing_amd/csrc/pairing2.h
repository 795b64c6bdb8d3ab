// Two lanes per pairing (gfx950): the Fq12 arithmetic of the Miller loop and
// the final exponentiation distributed over an adjacent lane pair.
//
// Why: at the BASELINE batch (2^16 pairings) one pairing per lane is exactly
// one wave per SIMD, and a lone wave issues a VALU instruction only every
// 4 cycles (MI355X_MICROARCH.md, "vector-instruction ISSUE cost").  With two
// lanes per pairing the batch is two waves per SIMD (full issue rate) and
// every lane does about half the multiplications.
//
// Layout: lane 2j+r (role r = 0, 1) of a wave holds c_r, the r-th Fq6 half
// of every Fq12 value of pairing j (Fq12 = c0 + c1 w, fq12.rs:9-12).  Both
// lanes run the same instruction stream (SIMT); what differs per role is
// chosen with selects, and values cross between the two lanes with
// `v_mov_b32_dpp quad_perm:[1,0,3,2]` (full-rate VALU, no LDS).
//
// Every function computes the same field values as the reference routine it
// cites, so outputs stay bit-exact (Fq12 values are canonical; G2 Jacobian
// coordinates and line coefficients follow mod.rs:176-245 value for value).
#pragma once
#include "pairing.h"

namespace pa {

// ---- lane-pair plumbing ----
PA_DEV uint32_t pair_swap_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);
}
PA_DEV void pswap(Fq& r, const Fq& a) {
#pragma unroll
    for (int i = 0; i < 12; i++) r.w[i] = pair_swap_u32(a.w[i]);
}
PA_DEV void pswap(Fq2& r, const Fq2& a) { pswap(r.c0, a.c0); pswap(r.c1, a.c1); }
PA_DEV void pswap(Fq6& r, const Fq6& a) { pswap(r.c0, a.c0); pswap(r.c1, a.c1); pswap(r.c2, a.c2); }

// sel(r, a, b) = r ? b : a  (per dword v_cndmask)
PA_DEV void sel(Fq& o, bool r, const Fq& a, const Fq& b) {
#pragma unroll
    for (int i = 0; i < 12; i++) o.w[i] = r ? b.w[i] : a.w[i];
}
PA_DEV void sel(Fq2& o, bool r, const Fq2& a, const Fq2& b) { sel(o.c0, r, a.c0, b.c0); sel(o.c1, r, a.c1, b.c1); }
PA_DEV void sel(Fq6& o, bool r, const Fq6& a, const Fq6& b) {
    sel(o.c0, r, a.c0, b.c0);
    sel(o.c1, r, a.c1, b.c1);
    sel(o.c2, r, a.c2, b.c2);
}

// ---- distributed Fq12 arithmetic (x, y, z: this lane's half) ----

// Fq12::mul_assign, fq12.rs:116-130 (Karatsuba over Fq6).
// Role 0 computes aa = x0*y0, role 1 bb = x1*y1 (6 Fq2 muls each); the cross
// product (x0+x1)(y0+y1) is split 3 + 3 over its six Karatsuba Fq2 products
// (fq6.rs:199-248).  9 Fq2 multiplications per lane instead of 18.
PA_NOINLINE void mul2(Fq6& z, const Fq6& x, const Fq6& y, bool r) {
    Fq6 P, S, T, t;
    mul(P, x, y);
    pswap(t, x);
    add(S, x, t);
    pswap(t, y);
    add(T, y, t);
    Fq2 u, v, p0, p1, p2, q0, q1, q2, a, b;
    add(a, S.c1, S.c2); add(b, T.c1, T.c2);
    sel(u, r, S.c0, a); sel(v, r, T.c0, b);
    mul(p0, u, v);
    add(a, S.c0, S.c2); add(b, T.c0, T.c2);
    sel(u, r, S.c1, a); sel(v, r, T.c1, b);
    mul(p1, u, v);
    add(a, S.c0, S.c1); add(b, T.c0, T.c1);
    sel(u, r, S.c2, a); sel(v, r, T.c2, b);
    mul(p2, u, v);
    pswap(q0, p0); pswap(q1, p1); pswap(q2, p2);
    Fq2 a_a, b_b, c_c, t1, t2, t3;
    sel(a_a, r, p0, q0); sel(b_b, r, p1, q1); sel(c_c, r, p2, q2);
    sel(t1, r, q0, p0); sel(t3, r, q1, p1); sel(t2, r, q2, p2);
    Fq6 C;
    sub(t1, t1, b_b); sub(t1, t1, c_c); mul_by_nonresidue(t1, t1); add(C.c0, t1, a_a);
    sub(t3, t3, a_a); add(t3, t3, b_b); sub(C.c2, t3, c_c);
    sub(t2, t2, a_a); sub(t2, t2, b_b); mul_by_nonresidue(c_c, c_c); add(C.c1, t2, c_c);
    Fq6 Po, z0, z1;
    pswap(Po, P);
    mul_by_nonresidue(z0, Po);
    add(z0, z0, P);       // role 0: aa + v*bb
    sub(z1, C, P);
    sub(z1, z1, Po);      // role 1: cross - aa - bb
    sel(z, r, z0, z1);
}

// Fq12::square, fq12.rs:99-114: role 0 computes ab = x0*x1, role 1 computes
// (x0 + v x1)(x0 + x1); one Fq6 multiply per lane instead of two.
PA_NOINLINE void sqr2(Fq6& z, const Fq6& x, bool r) {
    Fq6 xo, vx, a, b, t, p, po, z0, z1;
    pswap(xo, x);
    mul_by_nonresidue(vx, x);
    add(t, xo, vx);
    sel(a, r, x, t);
    add(t, xo, x);
    sel(b, r, xo, t);
    mul(p, a, b);
    pswap(po, p);              // role 0 receives (x0+vx1)(x0+x1), role 1 receives ab
    mul_by_nonresidue(vx, p);
    sub(z0, po, p);
    sub(z0, z0, vx);           // role 0: c0 = D - ab - v ab
    dbl(z1, po);               // role 1: c1 = 2 ab
    sel(z, r, z0, z1);
}

// Granger-Scott squaring in the cyclotomic subgroup.  The three Fq4
// components (a0,b1), (b0,a2), (a1,b2) each have one element on each lane.
// Per component (x, y): P = x*y (role 1), Q = (x+y)(x+xi y) (role 0); then
// x^2 + xi y^2 = Q - (1+xi) P and 2xy = 2P.  3 Fq2 multiplications per lane.
PA_NOINLINE void cyc_sqr2(Fq6& z, const Fq6& x, bool r) {
    // own element of components A, B, C: role 0 (a0, a2, a1), role 1 (b1, b0, b2)
    // Output slot of component k: role 0 -> k, role 1 -> k+1 (mod 3); the term
    // 2*own subtracted/added there is this lane's own element of that slot.
    Fq2 E[3], own[3], outs[3];
    sel(E[0], r, x.c0, x.c1);
    sel(E[1], r, x.c2, x.c0);
    sel(E[2], r, x.c1, x.c2);
    own[0] = E[0];
    sel(own[1], r, x.c1, x.c2);
    sel(own[2], r, x.c2, x.c0);
#pragma unroll
    for (int k = 0; k < 3; k++) {
        Fq2 F, X, Y, s, t, op1, op2, prod, other, a, b;
        pswap(F, E[k]);
        // component (x, y): A = (a0, b1) and C = (a1, b2) have x on role 0; B = (b0, a2) has x on role 1
        const bool x_on_role1 = (k == 1);
        sel(X, r != x_on_role1, E[k], F);
        sel(Y, r != x_on_role1, F, E[k]);
        add(s, E[k], F);                       // x + y
        mul_by_nonresidue(t, Y);
        add(t, t, X);                          // x + xi y
        sel(op1, r, s, X);
        sel(op2, r, t, Y);
        mul(prod, op1, op2);                   // role 0: Q, role 1: P
        pswap(other, prod);                    // role 0 receives P
        // role 0: 3 (Q - (1+xi) P) - 2 own
        mul_by_nonresidue(a, other);
        add(a, a, other);
        sub(a, prod, a);
        dbl(b, a);
        add(a, a, b);
        dbl(b, own[k]);
        sub(a, a, b);
        // role 1: 3 * 2 * m * P + 2 own, m = xi for component C
        Fq2 c, d;
        dbl(c, prod);
        if (k == 2) mul_by_nonresidue(c, c);
        dbl(d, c);
        add(c, c, d);
        dbl(d, own[k]);
        add(c, c, d);
        sel(outs[k], r, a, c);
    }
    // output slots: role 0 A->c0, B->c1, C->c2; role 1 A->c1, B->c2, C->c0
    sel(z.c0, r, outs[0], outs[2]);
    sel(z.c1, r, outs[1], outs[0]);
    sel(z.c2, r, outs[2], outs[1]);
}

// conjugate (fq12.rs:30-32): role 1 negates
PA_DEV void conj2(Fq6& z, const Fq6& x, bool r) {
    Fq6 n;
    neg(n, x);
    sel(z, r, x, n);
}

// Fq12::frobenius_map (fq12.rs:90-97)
PA_NOINLINE void frob2(Fq6& z, const Fq6& x, int power, bool r) {
    Fq6 t;
    frobenius_map(t, x, power);
    Fq2 k, one2;
    load_fq2_const(k, FROB_FQ12_C1[power % 12]);
    one(one2);
    sel(k, r, one2, k);
    mul(z.c0, t.c0, k);
    mul(z.c1, t.c1, k);
    mul(z.c2, t.c2, k);
}

// Fq12::inverse (fq12.rs:132-148); the Fq6 inversion is done by both lanes.
PA_NOINLINE bool inv2(Fq6& z, const Fq6& x, bool r) {
    Fq6 s, so, d, vs, t;
    sqr(s, x);                 // role 0: c0^2, role 1: c1^2
    pswap(so, s);
    Fq6 c0s, c1s;
    sel(c0s, r, s, so);
    sel(c1s, r, so, s);
    mul_by_nonresidue(vs, c1s);
    sub(d, c0s, vs);
    const bool ok = inverse(t, d);
    mul(s, x, t);
    conj2(z, s, r);
    return ok;
}

// ---- line functions (two lanes, R replicated on both) ----

// doubling_step, mod.rs:176-245: the same field values, with the eight
// squarings and three products spread over the pair (2+2 squarings and 2
// products per lane).
PA_NOINLINE void doubling_step2(EllCoeff& out, Jac<Fq2>& R, bool r) {
    Fq2 a1, a2, s1, s2, o1, o2, t, zy;
    sel(a1, r, R.x, R.y);
    add(zy, R.z, R.y);
    sel(a2, r, R.z, zy);
    sqr(s1, a1);
    sqr(s2, a2);
    pswap(o1, s1);
    pswap(o2, s2);
    Fq2 tmp0, tmp1, zsq, zy2;
    sel(tmp0, r, s1, o1);   // x^2
    sel(tmp1, r, o1, s1);   // y^2
    sel(zsq, r, s2, o2);    // z^2
    sel(zy2, r, o2, s2);    // (z+y)^2
    Fq2 tmp4, b1, b2, u1;
    dbl(tmp4, tmp0);
    add(tmp4, tmp4, tmp0);  // 3 x^2
    sel(b1, r, tmp1, tmp4);
    add(t, tmp1, R.x);
    add(u1, R.x, tmp4);
    sel(b2, r, t, u1);
    sqr(s1, b1);
    sqr(s2, b2);
    pswap(o1, s1);
    pswap(o2, s2);
    Fq2 tmp2, tmp3, tmp5, tmp6;
    sel(tmp2, r, s1, o1);   // y^4
    sel(tmp3, r, s2, o2);   // (y^2 + x)^2
    sel(tmp5, r, o1, s1);   // (3x^2)^2
    sel(tmp6, r, o2, s2);   // (x + 3x^2)^2
    sub(tmp3, tmp3, tmp0);
    sub(tmp3, tmp3, tmp2);
    dbl(tmp3, tmp3);
    Fq2 rx, rz;
    sub(rx, tmp5, tmp3);
    sub(rx, rx, tmp3);
    sub(rz, zy2, tmp1);
    sub(rz, rz, zsq);
    // products: role 0 (tmp3 - rx) * tmp4, role 1 rz * zsq; both tmp4 * zsq
    Fq2 m1, n1, p1, p2, q1;
    sub(t, tmp3, rx);
    sel(m1, r, t, rz);
    sel(n1, r, tmp4, zsq);
    mul(p1, m1, n1);
    mul(p2, tmp4, zsq);
    pswap(q1, p1);
    Fq2 ry_p, c0_p;
    sel(ry_p, r, p1, q1);
    sel(c0_p, r, q1, p1);
    dbl(tmp2, tmp2);
    dbl(tmp2, tmp2);
    dbl(tmp2, tmp2);
    Fq2 ry;
    sub(ry, ry_p, tmp2);
    // coefficients (tmp0', tmp3', tmp6') of mod.rs:226-244
    dbl(out.c1, p2);
    neg(out.c1, out.c1);
    sub(tmp6, tmp6, tmp0);
    sub(tmp6, tmp6, tmp5);
    dbl(tmp1, tmp1);
    dbl(tmp1, tmp1);
    sub(out.c2, tmp6, tmp1);
    dbl(out.c0, c0_p);
    R.x = rx;
    R.y = ry;
    R.z = rz;
}

// ell (mod.rs:57-69) + Fq12::mul_by_014 (fq12.rs:34-48) on the pair:
// role 0 scales c0 by P.y, role 1 scales c1 by P.x; the sparse product is
// own = half.mul_by_01(role 0: (c2, c1 x) ; role 1: (0, c0 y)) -- the latter
// equals mul_by_1(c0 y), fq6.rs:40-66 -- plus the Karatsuba cross term
// (x0+x1).mul_by_01(c2, c1x + c0y) split 3 + 3 over its five products.
PA_NOINLINE void ell2(Fq6& f, const EllCoeff& c, const Fq& px, const Fq& py, bool r) {
    Fq2 m, prod, other, c1x, c0y;
    sel(m, r, c.c0, c.c1);
    Fq s;
    sel(s, r, py, px);
    mul_by_fq(prod, m, s);
    pswap(other, prod);
    sel(c0y, r, prod, other);
    sel(c1x, r, other, prod);
    // own product
    Fq2 d0, d1, zero2;
    zero(zero2);
    sel(d0, r, c.c2, zero2);
    sel(d1, r, c1x, c0y);
    Fq6 P;
    mul_by_01(P, f, d0, d1);
    // cross term
    Fq6 S, t;
    pswap(t, f);
    add(S, f, t);
    Fq2 o, co, u, v, a;
    add(o, c1x, c0y);
    add(co, c.c2, o);
    Fq2 p0, p1, p2, q0, q1, q2;
    // slots: role 0 (s0*c0, s1*o, o*(s1+s2)); role 1 (c0*(s0+s2), (c0+o)*(s0+s1), dup)
    add(a, S.c0, S.c2);
    sel(u, r, S.c0, a);
    sel(v, r, c.c2, c.c2);
    mul(p0, u, v);
    add(a, S.c0, S.c1);
    sel(u, r, S.c1, a);
    sel(v, r, o, co);
    mul(p1, u, v);
    add(a, S.c1, S.c2);
    sel(u, r, a, a);
    mul(p2, u, o);
    pswap(q0, p0); pswap(q1, p1); pswap(q2, p2);
    Fq2 a_a, b_b, t1, t2, t3;
    sel(a_a, r, p0, q0);
    sel(b_b, r, p1, q1);
    sel(t1, r, p2, q2);
    sel(t3, r, q0, p0);
    sel(t2, r, q1, p1);
    Fq6 C;
    sub(t1, t1, b_b); mul_by_nonresidue(t1, t1); add(C.c0, t1, a_a);
    sub(t3, t3, a_a); add(C.c2, t3, b_b);
    sub(t2, t2, a_a); sub(C.c1, t2, b_b);
    Fq6 Po, z0, z1;
    pswap(Po, P);
    mul_by_nonresidue(z0, Po);
    add(z0, z0, P);
    sub(z1, C, P);
    sub(z1, z1, Po);
    sel(f, r, z0, z1);
}

PA_DEV void one2(Fq6& f, bool r) {
    Fq6 o, z;
    one(o);
    zero(z);
    sel(f, r, o, z);
}

// Single-pair Miller loop (mod.rs:40-102) on a lane pair, prepare fused.
PA_NOINLINE void miller_loop2(Fq6& f, const Aff<Fq>& p, const Aff<Fq2>& q, bool r) {
    Jac<Fq2> R;
    R.x = q.x;
    R.y = q.y;
    one(R.z);
    one2(f, r);
    EllCoeff c;
#pragma unroll 1
    for (int bit = 61; bit >= 0; bit--) {
        doubling_step2(c, R, r);
        ell2(f, c, p.x, p.y, r);
        if (((kBlsX >> 1) >> bit) & 1) {  // wave-uniform
            addition_step(c, R, q.x, q.y);
            ell2(f, c, p.x, p.y, r);
        }
        sqr2(f, f, r);
    }
    doubling_step2(c, R, r);
    ell2(f, c, p.x, p.y, r);
    conj2(f, f, r);
    if (p.inf || q.inf) one2(f, r);
}

// exp_by_x (mod.rs:116-121) with cyclotomic squarings
PA_NOINLINE void exp_by_x2(Fq6& z, const Fq6& f, uint64_t x, bool r) {
    Fq6 res = f;
    const int top = 63 - __builtin_clzll(x);
#pragma unroll 1
    for (int bit = top - 1; bit >= 0; bit--) {
        cyc_sqr2(res, res, r);
        if ((x >> bit) & 1) mul2(res, res, f, r);
    }
    conj2(z, res, r);
}

// final_exponentiation (mod.rs:104-160) on a lane pair
PA_NOINLINE bool final_exponentiation2(Fq6& out, const Fq6& f, bool r) {
    Fq6 f1, f2, rr, y0, y1, y2, y3;
    conj2(f1, f, r);
    const bool ok = inv2(f2, f, r);
    mul2(rr, f1, f2, r);
    f2 = rr;
    frob2(rr, rr, 2, r);
    mul2(rr, rr, f2, r);

    uint64_t x = kBlsX;
    cyc_sqr2(y0, rr, r);
    exp_by_x2(y1, y0, x, r);
    x >>= 1;
    exp_by_x2(y2, y1, x, r);
    x <<= 1;
    conj2(y3, rr, r);
    mul2(y1, y1, y3, r);
    conj2(y1, y1, r);
    mul2(y1, y1, y2, r);
    exp_by_x2(y2, y1, x, r);
    exp_by_x2(y3, y2, x, r);
    conj2(y1, y1, r);
    mul2(y3, y3, y1, r);
    conj2(y1, y1, r);
    frob2(y1, y1, 3, r);
    frob2(y2, y2, 2, r);
    mul2(y1, y1, y2, r);
    exp_by_x2(y2, y3, x, r);
    mul2(y2, y2, y0, r);
    mul2(y2, y2, rr, r);
    mul2(y1, y1, y2, r);
    frob2(y2, y3, 1, r);
    mul2(y1, y1, y2, r);
    out = y1;
    return ok;
}

}  // namespace pa
