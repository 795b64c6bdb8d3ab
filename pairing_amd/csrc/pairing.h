// Device-side BLS12-381 pairing: G2 line precomputation, Miller loop and
// final exponentiation, one pairing per lane (gfx950).
//
//   doubling_step / addition_step   reference src/bls12_381/mod.rs:176-333
//   G2Prepared::from_affine         mod.rs:168-358  (68 line coefficients)
//   ell                             mod.rs:57-69
//   Bls12::miller_loop              mod.rs:40-102
//   Bls12::final_exponentiation     mod.rs:104-160
//
// Bit-exactness: line coefficients depend on the Jacobian history of R, so
// the two steps below compute the reference's exact field-value sequence.
// The Miller-loop output and the final exponentiation output are field
// values, so their internal arithmetic (e.g. cyclotomic squaring inside
// exp_by_x) may differ from the reference while the bits stay identical.
#pragma once
#include "curve.h"

namespace pa {

constexpr uint64_t kBlsX = 0xd201000000010000ULL;  // |x|, x < 0 (mod.rs:23-25)
constexpr int kNumCoeffs = 68;                      // 62 doubling + 5 addition + 1 final doubling

struct EllCoeff {
    Fq2 c0, c1, c2;
};

// doubling_step, mod.rs:176-245 (Algorithm 26, eprint 2010/354)
PA_NOINLINE void doubling_step(EllCoeff& out, Jac<Fq2>& r) {
    Fq2 tmp0, tmp1, tmp2, tmp3, tmp4, tmp5, tmp6, zsquared;
    sqr(tmp0, r.x);
    sqr(tmp1, r.y);
    sqr(tmp2, tmp1);
    add(tmp3, tmp1, r.x);
    sqr(tmp3, tmp3);
    sub(tmp3, tmp3, tmp0);
    sub(tmp3, tmp3, tmp2);
    dbl(tmp3, tmp3);
    dbl(tmp4, tmp0);
    add(tmp4, tmp4, tmp0);
    add(tmp6, r.x, tmp4);
    sqr(tmp5, tmp4);
    sqr(zsquared, r.z);

    sub(r.x, tmp5, tmp3);
    sub(r.x, r.x, tmp3);
    add(r.z, r.z, r.y);
    sqr(r.z, r.z);
    sub(r.z, r.z, tmp1);
    sub(r.z, r.z, zsquared);
    sub(r.y, tmp3, r.x);
    mul(r.y, r.y, tmp4);
    dbl(tmp2, tmp2);
    dbl(tmp2, tmp2);
    dbl(tmp2, tmp2);
    sub(r.y, r.y, tmp2);

    mul(tmp3, tmp4, zsquared);
    dbl(tmp3, tmp3);
    neg(tmp3, tmp3);
    sqr(tmp6, tmp6);
    sub(tmp6, tmp6, tmp0);
    sub(tmp6, tmp6, tmp5);
    dbl(tmp1, tmp1);
    dbl(tmp1, tmp1);
    sub(tmp6, tmp6, tmp1);
    mul(tmp0, r.z, zsquared);
    dbl(tmp0, tmp0);

    out.c0 = tmp0;
    out.c1 = tmp3;
    out.c2 = tmp6;
}

// addition_step, mod.rs:247-333 (Algorithm 27, eprint 2010/354)
PA_NOINLINE void addition_step(EllCoeff& out, Jac<Fq2>& r, const Fq2& qx, const Fq2& qy) {
    Fq2 zsquared, ysquared, t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10, ztsquared;
    sqr(zsquared, r.z);
    sqr(ysquared, qy);
    mul(t0, zsquared, qx);
    add(t1, qy, r.z);
    sqr(t1, t1);
    sub(t1, t1, ysquared);
    sub(t1, t1, zsquared);
    mul(t1, t1, zsquared);
    sub(t2, t0, r.x);
    sqr(t3, t2);
    dbl(t4, t3);
    dbl(t4, t4);
    mul(t5, t4, t2);
    sub(t6, t1, r.y);
    sub(t6, t6, r.y);
    mul(t9, t6, qx);
    mul(t7, t4, r.x);

    sqr(r.x, t6);
    sub(r.x, r.x, t5);
    sub(r.x, r.x, t7);
    sub(r.x, r.x, t7);
    add(r.z, r.z, t2);
    sqr(r.z, r.z);
    sub(r.z, r.z, zsquared);
    sub(r.z, r.z, t3);
    add(t10, qy, r.z);
    sub(t8, t7, r.x);
    mul(t8, t8, t6);
    mul(t0, r.y, t5);
    dbl(t0, t0);
    sub(r.y, t8, t0);

    sqr(t10, t10);
    sub(t10, t10, ysquared);
    sqr(ztsquared, r.z);
    sub(t10, t10, ztsquared);
    dbl(t9, t9);
    sub(t9, t9, t10);
    dbl(t10, r.z);
    neg(t6, t6);
    dbl(t1, t6);

    out.c0 = t10;
    out.c1 = t1;
    out.c2 = t9;
}

// ell, mod.rs:57-69: f.mul_by_014(c2, c1 * P.x, c0 * P.y)
PA_DEV void ell(Fq12& f, const EllCoeff& c, const Fq& px, const Fq& py) {
    Fq2 a, b;
    mul_by_fq(a, c.c0, py);
    mul_by_fq(b, c.c1, px);
    mul_by_014(f, f, c.c2, b, a);
}

// ---- final exponentiation ----
// Granger-Scott squaring in the cyclotomic subgroup (f^(q^6+1)(q^2+1) = ...
// lies there after the easy part).  Same value as Fq12::square for such f.
// f = (g0 + g1 w) with g0=(a0,a1,a2), g1=(b0,b1,b2); pairs (a0,b1), (b0,a2), (a1,b2)
// are the three Fq4 = Fq2[s]/(s^2 - xi) components.
PA_DEV void fq4_sqr(Fq2& r0, Fq2& r1, const Fq2& a, const Fq2& b) {
    // (a + b s)^2 = (a^2 + xi b^2) + ((a+b)^2 - a^2 - b^2) s
    Fq2 t0, t1, t2;
    sqr(t0, a);
    sqr(t1, b);
    add(t2, a, b);
    sqr(t2, t2);
    sub(t2, t2, t0);
    sub(r1, t2, t1);
    mul_by_nonresidue(t1, t1);
    add(r0, t1, t0);
}
PA_NOINLINE void cyclotomic_sqr(Fq12& r, const Fq12& f) {
    const Fq2& a0 = f.c0.c0; const Fq2& a1 = f.c0.c1; const Fq2& a2 = f.c0.c2;
    const Fq2& b0 = f.c1.c0; const Fq2& b1 = f.c1.c1; const Fq2& b2 = f.c1.c2;
    Fq2 t0, t1, t2, t3, t4, t5, tmp;
    fq4_sqr(t0, t1, a0, b1);   // A = a0 + b1 s
    fq4_sqr(t2, t3, b0, a2);   // B = b0 + a2 s
    fq4_sqr(t4, t5, a1, b2);   // C = a1 + b2 s
    Fq12 o;
    // c0.c0 = 3 t0 - 2 a0
    sub(tmp, t0, a0); dbl(tmp, tmp); add(o.c0.c0, tmp, t0);
    // c0.c1 = 3 t2 - 2 a1
    sub(tmp, t2, a1); dbl(tmp, tmp); add(o.c0.c1, tmp, t2);
    // c0.c2 = 3 t4 - 2 a2
    sub(tmp, t4, a2); dbl(tmp, tmp); add(o.c0.c2, tmp, t4);
    // c1.c0 = 3 xi t5 + 2 b0
    Fq2 t5x;
    mul_by_nonresidue(t5x, t5);
    add(tmp, t5x, b0); dbl(tmp, tmp); add(o.c1.c0, tmp, t5x);
    // c1.c1 = 3 t1 + 2 b1
    add(tmp, t1, b1); dbl(tmp, tmp); add(o.c1.c1, tmp, t1);
    // c1.c2 = 3 t3 + 2 b2
    add(tmp, t3, b2); dbl(tmp, tmp); add(o.c1.c2, tmp, t3);
    r = o;
}

}  // namespace pa
